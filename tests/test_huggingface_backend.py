"""`backend: huggingface` (langchain.go): chat / completion requests go to the Hugging Face
Inference API -- here a local test double that records what it receives."""
import json
import socket
import threading
import time

import pytest


@pytest.fixture()
def hf_double():
    import uvicorn
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse
    seen = []
    app = FastAPI()

    @app.post("/models/{org}/{name}")
    async def gen(org: str, name: str, request: Request):
        body = await request.json()
        seen.append({"model": f"{org}/{name}", "auth": request.headers.get("authorization"), "body": body})
        if org == "broken":
            return JSONResponse({"error": "Model is overloaded"}, status_code=503)
        return [{"generated_text": "Paris is the capital.\nQuestion: more"}]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    deadline = time.time() + 20
    while not srv.started and time.time() < deadline:
        time.sleep(0.05)
    yield f"http://127.0.0.1:{port}", seen
    srv.should_exit = True
    th.join(5)


def _app(tmp_path, model):
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    (tmp_path / "m").mkdir(exist_ok=True)
    ac = ApplicationConfig(models_path=str(tmp_path / "m"), upload_dir=str(tmp_path / "up"),
                           config_dir=str(tmp_path / "cfg"), image_dir=str(tmp_path / "img"),
                           audio_dir=str(tmp_path / "aud"))
    ac.engine_mode = "inprocess"
    st = AppState(ac)
    bc = BackendConfig({"name": "hf", "backend": "huggingface", "parameters": {"model": model, "temperature": 0.3},
                        "stopwords": ["\nQuestion:"], "template": {"chat": "{{.Input}}\nAnswer:"}})
    bc.set_defaults()
    st.configs.add(bc)
    return create_app(st)


def test_chat_and_completion_through_hf_api(tmp_path, hf_double, monkeypatch):
    from fastapi.testclient import TestClient
    url, seen = hf_double
    monkeypatch.setenv("HF_INFERENCE_ENDPOINT", url)
    monkeypatch.setenv("HUGGINGFACEHUB_API_TOKEN", "hf_test")
    with TestClient(_app(tmp_path, "tiiuae/falcon-7b-instruct")) as c:
        r = c.post("/v1/chat/completions", json={"model": "hf", "max_tokens": 20,
                                                 "messages": [{"role": "user", "content": "capital of France?"}]})
        assert r.status_code == 200, r.text
        assert r.json()["choices"][0]["message"]["content"] == "Paris is the capital."
        got = seen[-1]
        assert got["model"] == "tiiuae/falcon-7b-instruct" and got["auth"] == "Bearer hf_test"
        p = got["body"]["parameters"]
        assert p["max_new_tokens"] == 20 and abs(p["temperature"] - 0.3) < 1e-6 and p["stop"] == ["\nQuestion:"]
        assert got["body"]["inputs"].endswith("Answer:") and got["body"]["options"] == {"wait_for_model": True}
        # streaming: the whole completion arrives as one delta (langchain.go PredictStream)
        with c.stream("POST", "/v1/completions", json={"model": "hf", "prompt": "hi", "stream": True}) as s:
            chunks = [json.loads(line[6:]) for line in s.iter_lines() if line.startswith("data: {")]
        text = "".join(ch["choices"][0].get("text", "") for ch in chunks)
        assert text == "Paris is the capital."


def test_missing_token_and_api_error(tmp_path, hf_double, monkeypatch):
    from fastapi.testclient import TestClient
    url, _ = hf_double
    monkeypatch.setenv("HF_INFERENCE_ENDPOINT", url)
    monkeypatch.delenv("HUGGINGFACEHUB_API_TOKEN", raising=False)
    with TestClient(_app(tmp_path, "org/m"), raise_server_exceptions=False) as c:
        r = c.post("/v1/completions", json={"model": "hf", "prompt": "x"})
        assert r.status_code == 500 and "no huggingface token" in r.text
    monkeypatch.setenv("HUGGINGFACEHUB_API_TOKEN", "t")
    with TestClient(_app(tmp_path, "broken/m"), raise_server_exceptions=False) as c:
        r = c.post("/v1/completions", json={"model": "hf", "prompt": "x"})
        assert r.status_code == 500 and "503" in r.text
