"""`run --p2p`: network token, announce to federated balancers, node census with the 40-s
liveness rule, `/api/p2p`, `/api/p2p/token` and the `/p2p` page (core/p2p, endpoints/localai/p2p.go)."""
import base64
import socket
import threading
import time

from localai_amd.gateway.explorer import decode_network_token, make_network_token
from localai_amd.gateway.p2p import NodeData, P2PNode, advertise_url, network_service_id


def test_generated_token_names_this_instance():
    n = P2PNode("", "lab", "http://me:8080", probe=lambda u, t: False)
    net = decode_network_token(n.token)
    assert net == {"network_id": "lab", "federated": [], "workers": ["http://me:8080"]}
    n.census_once()
    nodes = n.nodes()
    assert [d["ID"] for d in nodes["nodes"]] == ["http://me:8080"] and nodes["federated_nodes"] == []
    assert nodes["nodes"][0]["ServiceID"] == "lab_worker" == network_service_id("lab", "worker")


def test_join_announces_and_reads_balancer():
    announced, fetched = [], []
    tok = make_network_token(federated=["http://lb:9000"], workers=["http://peer:1"], network_id="")

    def get_json(url, timeout):
        fetched.append(url)
        return [{"url": "http://me:8080", "healthy": True}, {"url": "http://sick:1", "healthy": False}]
    n = P2PNode(tok, "", "http://me:8080", get_json=get_json, probe=lambda u, t: u == "http://peer:1/readyz",
                announce=lambda b, me, t: announced.append((b, me)) or True)
    n.census_once()
    assert announced == [("http://lb:9000", "http://me:8080")]
    assert fetched == ["http://lb:9000/federated/workers"]
    got = n.nodes()
    assert sorted(d["ID"] for d in got["nodes"]) == ["http://me:8080", "http://peer:1"]
    assert [d["ID"] for d in got["federated_nodes"]] == ["http://lb:9000"]


def test_liveness_rule():
    now = time.time()
    assert NodeData("a", "a", LastSeen=now - 10).is_online(now)
    assert not NodeData("a", "a", LastSeen=now - 41).is_online(now)


def test_advertise_url(monkeypatch):
    monkeypatch.delenv("LOCALAI_ADVERTISE_URL", raising=False)
    assert advertise_url("127.0.0.1:9090") == "http://127.0.0.1:9090"
    assert advertise_url(":8080") == f"http://{socket.gethostname()}:8080"
    monkeypatch.setenv("LOCALAI_ADVERTISE_URL", "http://node7:80/")
    assert advertise_url(":8080") == "http://node7:80"


def test_p2p_routes_in_app(tmp_path, monkeypatch):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    monkeypatch.setenv("LOCALAI_ADVERTISE_URL", "http://127.0.0.1:1")
    ac = ApplicationConfig(models_path=str(tmp_path / "m"), upload_dir=str(tmp_path / "up"),
                           config_dir=str(tmp_path / "cfg"), image_dir=str(tmp_path / "img"),
                           audio_dir=str(tmp_path / "aud"))
    (tmp_path / "m").mkdir()
    ac.p2p, ac.p2p_network_id = True, "net1"
    app = create_app(AppState(ac))
    with TestClient(app) as c:
        tok = c.get("/api/p2p/token").text
        assert decode_network_token(tok)["workers"] == ["http://127.0.0.1:1"]
        deadline = time.time() + 10
        while not c.get("/api/p2p").json()["nodes"] and time.time() < deadline:
            time.sleep(0.05)
        j = c.get("/api/p2p").json()
        assert set(j) == {"nodes", "federated_nodes"} and j["nodes"][0]["ID"] == "http://127.0.0.1:1"
        assert "1</b>/<b>1" in c.get("/p2p/ui/workers-stats").text
        assert "online" in c.get("/p2p/ui/workers").text
        page = c.get("/p2p")
        assert page.status_code == 200 and "Network token" in page.text


def test_p2p_routes_absent_without_flag(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    (tmp_path / "m").mkdir()
    ac = ApplicationConfig(models_path=str(tmp_path / "m"), upload_dir=str(tmp_path / "up"),
                           config_dir=str(tmp_path / "cfg"), image_dir=str(tmp_path / "img"),
                           audio_dir=str(tmp_path / "aud"))
    with TestClient(create_app(AppState(ac))) as c:
        assert c.get("/api/p2p/token").status_code == 404


def test_join_real_balancer_over_http():
    """A balancer (gateway/federated.py) named by a URL token learns this instance's URL from the
    announce, then routes to it."""
    import uvicorn

    from localai_amd.gateway.federated import FederatedBalancer, create_federated_app
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    bal = FederatedBalancer([])
    srv = uvicorn.Server(uvicorn.Config(create_federated_app(bal), host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    try:
        deadline = time.time() + 20
        while not srv.started and time.time() < deadline:
            time.sleep(0.05)
        tok = base64.b64encode(f"http://127.0.0.1:{port}".encode()).decode()
        n = P2PNode(tok, "", "http://127.0.0.1:7", probe=lambda u, t: False)
        n.census_once()
        assert "http://127.0.0.1:7" in bal.workers
        assert [d["ID"] for d in n.nodes()["federated_nodes"]] == [f"http://127.0.0.1:{port}"]
    finally:
        srv.should_exit = True
        th.join(5)
