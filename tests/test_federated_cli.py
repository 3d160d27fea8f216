"""Federated load balancer, CLI parsing, startup (model install from file:// gallery, dynamic
config watcher) -- reference core/p2p/federated*.go, core/cli/*, core/startup/*."""
import json
import os
import threading
import time
import urllib.request

import yaml

from localai_amd import cli
from localai_amd.config.app_config import ApplicationConfig


def _serve(app):
    from localai_amd.gateway.native_server import NativeHTTPServer
    srv = NativeHTTPServer(app, "127.0.0.1", 0)
    threading.Thread(target=srv.run, daemon=True).start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 20:
        time.sleep(0.02)
    return srv


def test_federated_balancer_routes_and_streams():
    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse
    from localai_amd.gateway.federated import FederatedBalancer, create_federated_app

    def worker(tag):
        app = FastAPI()

        @app.get("/readyz")
        async def ready():
            return {}

        @app.post("/v1/echo")
        async def echo(req: dict):
            return {"worker": tag, "got": req}

        @app.get("/v1/stream")
        async def stream():
            async def gen():
                for i in range(3):
                    yield f"data: {tag}-{i}\n\n".encode()
            return StreamingResponse(gen(), media_type="text/event-stream")
        return _serve(app)
    w1, w2 = worker("a"), worker("b")
    bal = FederatedBalancer([f"http://127.0.0.1:{w1.port}", f"http://127.0.0.1:{w2.port}"])
    front = _serve(create_federated_app(bal))
    base = f"http://127.0.0.1:{front.port}"
    seen = set()
    for i in range(4):
        req = urllib.request.Request(base + "/v1/echo", data=json.dumps({"i": i}).encode(),
                                     headers={"content-type": "application/json"})
        r = json.loads(urllib.request.urlopen(req, timeout=20).read())
        assert r["got"] == {"i": i}
        seen.add(r["worker"])
    assert seen == {"a", "b"}  # least-used alternates between idle workers
    body = urllib.request.urlopen(base + "/v1/stream", timeout=20).read().decode()
    assert body.count("data:") == 3
    ws = json.loads(urllib.request.urlopen(base + "/federated/workers", timeout=20).read())
    assert len(ws) == 2 and sum(w["served"] for w in ws) == 5
    for s in (front, w1, w2):
        s.shutdown()


def test_cli_run_flags_and_env(monkeypatch):
    monkeypatch.setenv("LOCALAI_CONTEXT_SIZE", "1024")
    monkeypatch.setenv("THREADS", "3")
    ap = cli.build_parser()
    a = ap.parse_args(["run", "--models-path", "/tmp/m", "--api-keys", "k1,k2", "--cors",
                       "--external-grpc-backends", "whisper:127.0.0.1:9000", "--watchdog-idle-timeout", "2m",
                       "http://x/model.yaml"])
    c = cli.app_config_from_args(a)
    assert c.models_path == "/tmp/m" and c.api_keys == ["k1", "k2"] and c.cors is True
    assert c.context_size == 1024 and c.threads == 3
    assert c.external_grpc_backends == {"whisper": "127.0.0.1:9000"}
    assert c.watchdog_idle_timeout == 120.0 and c.model_urls[-1] == "http://x/model.yaml"


def test_startup_installs_gallery_model_and_watches_config(tmp_path):
    from localai_amd.startup import startup
    models, dyn = tmp_path / "models", tmp_path / "dyn"
    gal_dir = models / "gallery"  # file:// gallery resources must live under the models path
    gal_dir.mkdir(parents=True)
    (gal_dir / "weights.bin").write_bytes(b"\x00" * 16)
    cfg_file = gal_dir / "tiny.yaml"
    cfg_file.write_text(yaml.safe_dump({
        "name": "tiny", "config_file": yaml.safe_dump({"backend": "llama-cpp", "parameters": {"model": "weights.bin"},
                                                       "context_size": 256}),
        "files": [{"filename": "weights.bin", "uri": f"file://{gal_dir}/weights.bin"}],
        "prompt_templates": [{"name": "tiny-chat", "content": "{{.Input}}"}]}))
    index = gal_dir / "index.yaml"
    index.write_text(yaml.safe_dump([{"name": "tiny", "url": f"file://{cfg_file}"}]))
    app = ApplicationConfig(models_path=str(models), galleries=[{"name": "local", "url": f"file://{index}"}],
                            model_urls=["local@tiny"], dynamic_config_dir=str(dyn), dynamic_config_poll_interval=0.1,
                            image_dir=str(tmp_path / "i"), audio_dir=str(tmp_path / "a"),
                            upload_dir=str(tmp_path / "u"), config_dir=str(tmp_path / "c"))
    state = startup(app)
    assert (models / "weights.bin").exists() and (models / "tiny-chat.tmpl").exists()
    assert state.configs.get("tiny") is not None and state.configs.get("tiny").raw["context_size"] == 256
    (dyn / "api_keys.json").write_text(json.dumps(["dyn-key"]))
    t0 = time.time()
    while "dyn-key" not in app.api_keys and time.time() - t0 < 5:
        time.sleep(0.05)
    assert "dyn-key" in app.api_keys
    state.watcher.stop()


def test_util_hf_scan_uris_and_installed_gallery_models(tmp_path, capsys):
    """`util hf-scan` (core/cli/util.go:75-110): Hub scan verdicts via an injected fetch (no network)."""
    import pytest

    from localai_amd.utils.downloader import NonHuggingFaceFile, UnsafeFilesFound, hf_scan
    seen = []

    def fetch(url):
        seen.append(url)
        bad = "evil" in url
        return json.dumps({"repositoryId": url.split("/")[5], "hasUnsafeFile": bad, "scansDone": True,
                           "dangerousPickles": ["model.pkl"] if bad else []}).encode()

    ok = hf_scan("huggingface://TheBloke/good-GGUF/good.Q4_K_M.gguf", fetch=fetch)
    assert ok["scansDone"] and seen[-1] == "https://huggingface.co/api/models/TheBloke/good-GGUF/scan"
    with pytest.raises(UnsafeFilesFound) as ei:
        hf_scan("https://huggingface.co/someone/evil-repo/resolve/main/model.pkl", fetch=fetch)
    assert ei.value.result["dangerousPickles"] == ["model.pkl"]
    with pytest.raises(NonHuggingFaceFile):
        hf_scan("https://example.com/a/b/c.gguf", fetch=fetch)

    ns = cli.build_parser().parse_args(["util", "hf-scan", "huggingface://a/good/x.gguf",
                                        "hf://someone/evil/x.bin", "https://example.com/x"])
    assert cli._hf_scan(ns, fetch=fetch) == 1
    out = capsys.readouterr().out
    assert "known-vulnerable" in out and "evil" in out and "scan skipped" in out

    # no URIs: scan the files of installed gallery models only
    models = tmp_path / "models"
    models.mkdir()
    idx = models / "index.yaml"  # file:// galleries must live under the models path
    idx.write_text(yaml.safe_dump([
        {"name": "inst-evil", "files": [{"filename": "m.bin", "uri": "huggingface://x/evil/m.bin"}]},
        {"name": "not-installed", "files": [{"filename": "m.bin", "uri": "huggingface://x/evil2/m.bin"}]},
        {"name": "inst-good", "files": [{"filename": "g.gguf", "uri": "huggingface://x/good/g.gguf"}]}]))
    (models / "inst-evil.yaml").write_text("name: inst-evil\n")
    (models / "inst-good.yaml").write_text("name: inst-good\n")
    gal = json.dumps([{"name": "local", "url": "file://" + str(idx)}])
    ns = cli.build_parser().parse_args(["util", "hf-scan", "--models-path", str(models), "--galleries", gal])
    assert cli._hf_scan(ns, fetch=fetch) == 1
    out = capsys.readouterr().out
    assert "inst-evil" in out and "not-installed" not in out and "inst-good" not in out
