"""Network explorer (`core/explorer/database_test.go` cases + discovery and HTTP routes)."""
import base64
import json
import threading
import time

import pytest

from localai_amd.gateway.explorer import (ClusterData, Database, DiscoveryServer, TokenData,
                                          create_explorer_app, decode_network_token,
                                          make_network_token, parse_duration)


def test_database_add_get_delete_persist(tmp_path):
    path = str(tmp_path / "explorer.json")
    db = Database(path)
    assert db.get("x") == (TokenData(), False)  # starts empty
    t = TokenData(name="n", description="d", Clusters=[ClusterData(["a"], "worker", "net")])
    db.set("tok", t)
    got, ok = db.get("tok")
    assert ok and got == t
    # a second handle on the same file (another process's view) sees the same data
    db2 = Database(path)
    assert db2.get("tok") == (t, True)
    assert db2.token_list() == ["tok"]
    db.delete("tok")
    assert db2.get("tok")[1] is False


def test_database_concurrent_writers(tmp_path):
    path = str(tmp_path / "explorer.json")
    dbs = [Database(path) for _ in range(4)]

    def put(i):
        for j in range(10):
            dbs[i].set(f"t{i}_{j}", TokenData(name=str(j)))
    th = [threading.Thread(target=put, args=(i,)) for i in range(4)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert len(Database(path).token_list()) == 40


def test_token_roundtrip_and_validation():
    tok = make_network_token(federated=["http://a:8080"], workers=["http://w1:8080"], network_id="lab")
    d = decode_network_token(tok)
    assert d == {"network_id": "lab", "federated": ["http://a:8080"], "workers": ["http://w1:8080"]}
    url_tok = base64.b64encode(b"http://lb:9000").decode()
    assert decode_network_token(url_tok)["federated"] == ["http://lb:9000"]
    for bad in ("not base64!!", base64.b64encode(b"{}").decode(), base64.b64encode(b"[1]").decode()):
        with pytest.raises(ValueError):
            decode_network_token(bad)


def test_parse_duration():
    assert parse_duration("2m") == 120
    assert parse_duration("1h30m") == 5400
    assert parse_duration("500ms") == 0.5
    assert parse_duration("7") == 7
    with pytest.raises(ValueError):
        parse_duration("3x")


def _fake_net(fed_workers, live):
    def fetch_json(url, timeout):
        if url in fed_workers:
            return 200, fed_workers[url]
        raise OSError("refused")

    def probe(url, timeout):
        return url in live
    return fetch_json, probe


def test_discovery_census_failures_and_removal(tmp_path):
    db = Database(str(tmp_path / "e.json"))
    good = make_network_token(federated=["http://lb:1"], workers=["http://w1:2", "http://w2:2"], network_id="n1")
    dead = make_network_token(workers=["http://gone:3"])
    db.set(good, TokenData(name="good", description="g"))
    db.set(dead, TokenData(name="dead", description="d"))
    fetch, probe = _fake_net({"http://lb:1/federated/workers": [
        {"url": "http://x:1", "healthy": True}, {"url": "http://y:1", "healthy": False}]},
        {"http://w1:2/readyz"})
    ds = DiscoveryServer(db, connection_timeout=5, error_threshold=2, fetch_json=fetch, probe=probe)
    ds.run_once()
    g, _ = db.get(good)
    assert g.Failures == 0
    assert [(c.Type, c.Workers, c.NetworkID) for c in g.Clusters] == [
        ("federated", ["http://x:1"], "n1"), ("worker", ["http://w1:2"], "n1")]
    assert db.get(dead)[0].Failures == 1
    ds.run_once()
    ds.run_once()  # 3 failures > threshold 2 -> removed
    assert not db.get(dead)[1]
    assert db.get(good)[1]


def test_discovery_recovers_failure_count(tmp_path):
    db = Database(str(tmp_path / "e.json"))
    tok = make_network_token(workers=["http://w:1"])
    db.set(tok, TokenData(name="a", description="b", Failures=2))
    live = set()
    ds = DiscoveryServer(db, 5, 3, fetch_json=lambda u, t: (404, None), probe=lambda u, t: u in live)
    live.add("http://w:1/readyz")
    ds.run_once()
    assert db.get(tok)[0].Failures == 0


def test_explorer_http_routes(tmp_path):
    from fastapi.testclient import TestClient
    db = Database(str(tmp_path / "e.json"))
    c = TestClient(create_explorer_app(db))
    assert "Version" in c.get("/", headers={"accept": "application/json"}).json()
    page = c.get("/", headers={"accept": "text/html"})
    assert page.status_code == 200 and "network explorer" in page.text
    tok = make_network_token(workers=["http://w:1"])
    assert c.post("/network/add", json={"token": tok, "name": "n"}).json() == {"error": "Description is required"}
    assert c.post("/network/add", json={"token": "@@", "name": "n", "description": "d"}).status_code == 400
    r = c.post("/network/add", json={"token": tok, "name": "<img src=x>", "description": "d"})
    assert r.json() == {"message": "Token added"}
    assert c.post("/network/add", json={"token": tok, "name": "n", "description": "d"}).json()["error"] == \
        "Token already exists"
    assert c.get("/networks").json() == []  # no online workers yet
    db.set(tok, TokenData(name="<img src=x>", description="d", Clusters=[ClusterData(["http://w:1"], "worker")]))
    nets = c.get("/networks").json()
    assert len(nets) == 1 and nets[0]["token"] == tok and nets[0]["Clusters"][0]["Workers"] == ["http://w:1"]
    # names reach the page only through textContent, never as markup
    assert "<img src=x>" not in page.text


def test_discovery_against_live_federated_balancer(tmp_path):
    """End to end over real sockets: a federated balancer (gateway/federated.py) with one live
    worker; the explorer's census reads its /federated/workers list."""
    import socket

    import uvicorn
    from fastapi import FastAPI

    from localai_amd.gateway.federated import FederatedBalancer, create_federated_app

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    worker = FastAPI()

    @worker.get("/readyz")
    def readyz():
        return "OK"
    wp, lp = free_port(), free_port()
    wurl = f"http://127.0.0.1:{wp}"
    servers = [uvicorn.Server(uvicorn.Config(worker, host="127.0.0.1", port=wp, log_level="error")),
               uvicorn.Server(uvicorn.Config(create_federated_app(FederatedBalancer([wurl])), host="127.0.0.1",
                                             port=lp, log_level="error"))]
    ths = [threading.Thread(target=s.run, daemon=True) for s in servers]
    try:
        # worker first: the balancer's health loop probes it as soon as the balancer starts
        for srv, t in zip(servers, ths):
            t.start()
            deadline = time.time() + 20
            while not srv.started and time.time() < deadline:
                time.sleep(0.05)
        db = Database(str(tmp_path / "e.json"))
        tok = base64.b64encode(f"http://127.0.0.1:{lp}".encode()).decode()
        db.set(tok, TokenData(name="lab", description="one node"))
        DiscoveryServer(db, connection_timeout=10).run_once()
        data, _ = db.get(tok)
        assert data.Failures == 0
        assert data.Clusters == [ClusterData([wurl], "federated", "")]
    finally:
        for s in servers:
            s.should_exit = True
        [t.join(5) for t in ths]


def test_cli_explorer_only_sync(tmp_path, monkeypatch):
    from localai_amd import cli
    path = str(tmp_path / "e.json")
    Database(path).set(make_network_token(workers=["http://127.0.0.1:9/"]), TokenData(name="a", description="b"))
    assert cli.main(["explorer", "--only-sync", "--pool-database", path, "--connection-timeout", "2s"]) == 0
    doc = json.load(open(path))
    assert list(doc.values())[0]["Failures"] == 1
