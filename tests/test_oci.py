"""oci:// and ollama:// model URIs against a local OCI registry double (token auth challenge,
manifest negotiation, image index, blob digests), layer unpacking rules, and resumed http(s)
downloads (Range) -- pkg/oci, pkg/downloader/uri.go, pkg/startup/model_preload.go."""
import gzip
import hashlib
import io
import json
import os
import socket
import tarfile
import threading
import time

import pytest

from localai_amd.utils import oci
from localai_amd.utils.downloader import download_file


def _tar(files, gz=True, extra=None):
    b = io.BytesIO()
    with tarfile.open(fileobj=b, mode="w") as tf:
        for name, data in files.items():
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
        for ti in extra or []:
            tf.addfile(ti)
    raw = b.getvalue()
    return gzip.compress(raw) if gz else raw


def _digest(b):
    return "sha256:" + hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def registry():
    import uvicorn
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, Response
    blobs, manifests = {}, {}
    evil = tarfile.TarInfo("../../escape.txt")
    evil.size = 0
    layer1 = _tar({"models/model.gguf": b"GGUF-weights", "models/old.txt": b"x"})
    layer2 = _tar({"models/.wh.old.txt": b"", "models/model.yaml": b"name: m\n"}, gz=False, extra=[evil])
    ollama_model = b"ollama-gguf-bytes" * 100
    for b in (layer1, layer2, ollama_model, b"{}"):
        blobs[_digest(b)] = b
    img = {"schemaVersion": 2, "mediaType": "application/vnd.oci.image.manifest.v1+json",
           "config": {"digest": _digest(b"{}"), "size": 2, "mediaType": "application/vnd.oci.image.config.v1+json"},
           "layers": [{"digest": _digest(layer1), "size": len(layer1), "mediaType": "application/vnd.oci.image.layer.v1.tar+gzip"},
                      {"digest": _digest(layer2), "size": len(layer2), "mediaType": "application/vnd.oci.image.layer.v1.tar"}]}
    img_b = json.dumps(img).encode()
    manifests[("org/models", _digest(img_b))] = img_b
    idx = {"schemaVersion": 2, "mediaType": "application/vnd.oci.image.index.v1+json",
           "manifests": [{"digest": "sha256:" + "0" * 64, "platform": {"os": "linux", "architecture": "arm64"}},
                         {"digest": _digest(img_b), "platform": {"os": "linux", "architecture": "amd64"}}]}
    manifests[("org/models", "v1")] = json.dumps(idx).encode()
    oll = {"schemaVersion": 2, "layers": [{"digest": _digest(b"{}"), "mediaType": "application/vnd.ollama.image.params"},
                                          {"digest": _digest(ollama_model), "mediaType": "application/vnd.ollama.image.model",
                                           "size": len(ollama_model)}]}
    manifests[("library/gemma", "2b")] = json.dumps(oll).encode()
    manifests[("acme/tiny", "latest")] = json.dumps(oll).encode()
    app = FastAPI()
    state = {"port": 0, "ranges": []}

    def authed(req):
        return req.headers.get("authorization") == "Bearer tok123"

    @app.get("/token")
    def token(scope: str = "", service: str = ""):
        assert scope.startswith("repository:") and service == "test"
        return {"token": "tok123"}

    @app.get("/v2/{repo:path}/manifests/{ref}")
    def manifest(repo: str, ref: str, request: Request):
        if not authed(request):
            return Response(status_code=401, headers={
                "WWW-Authenticate": f'Bearer realm="http://127.0.0.1:{state["port"]}/token",service="test"'})
        body = manifests.get((repo, ref))
        if body is None:
            return JSONResponse({"errors": []}, status_code=404)
        return Response(body, media_type=json.loads(body).get("mediaType", "application/vnd.oci.image.manifest.v1+json"))

    @app.get("/v2/{repo:path}/blobs/{digest}")
    def blob(repo: str, digest: str, request: Request):
        if not authed(request):
            return Response(status_code=401, headers={
                "WWW-Authenticate": f'Bearer realm="http://127.0.0.1:{state["port"]}/token",service="test"'})
        return Response(blobs[digest], media_type="application/octet-stream")

    payload = bytes(range(256)) * 64

    @app.get("/files/big.bin")
    def big(request: Request):
        rng = request.headers.get("range")
        state["ranges"].append(rng)
        if rng:
            start = int(rng.split("=")[1].split("-")[0])
            if start >= len(payload):
                return Response(status_code=416)
            return Response(payload[start:], status_code=206, media_type="application/octet-stream")
        return Response(payload, media_type="application/octet-stream")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    state["port"] = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=state["port"], log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    deadline = time.time() + 20
    while not srv.started and time.time() < deadline:
        time.sleep(0.05)
    yield f"127.0.0.1:{state['port']}", ollama_model, payload, state
    srv.should_exit = True
    th.join(5)


def test_parse_reference():
    assert oci.parse_reference("alpine") == ("registry-1.docker.io", "library/alpine", "latest")
    assert oci.parse_reference("quay.io/org/img:1.2") == ("quay.io", "org/img", "1.2")
    assert oci.parse_reference("localhost:5000/a/b@sha256:ab") == ("localhost:5000", "a/b", "sha256:ab")
    assert oci.parse_reference("docker.io/user/repo") == ("registry-1.docker.io", "user/repo", "latest")


def test_oci_image_unpacked_into_model_dir(registry, tmp_path):
    host, _, _, _ = registry
    dst = tmp_path / "models" / "org__models__v1"
    download_file(f"oci://{host}/org/models:v1", str(dst))
    root = tmp_path / "models"
    assert (root / "models" / "model.gguf").read_bytes() == b"GGUF-weights"
    assert (root / "models" / "model.yaml").exists()
    assert not (root / "models" / "old.txt").exists()          # whiteout of the lower layer's file
    assert not (tmp_path / "escape.txt").exists() and not (tmp_path.parent / "escape.txt").exists()


def test_ollama_model_blob(registry, tmp_path):
    host, model, _, _ = registry
    os.environ["LOCALAI_OLLAMA_REGISTRY"] = host
    try:
        p = download_file("ollama://gemma:2b", str(tmp_path / "gemma__2b"))
        assert open(p, "rb").read() == model
        p2 = download_file("ollama://acme/tiny", str(tmp_path / "acme__tiny"))  # namespace honoured
        assert open(p2, "rb").read() == model
    finally:
        del os.environ["LOCALAI_OLLAMA_REGISTRY"]


def test_startup_installs_ollama_uri(registry, tmp_path):
    from localai_amd.startup import install_models
    host, model, _, _ = registry
    os.environ["LOCALAI_OLLAMA_REGISTRY"] = host
    try:
        assert install_models([], str(tmp_path), ["ollama://gemma:2b"]) == []
        assert (tmp_path / "gemma__2b").read_bytes() == model
    finally:
        del os.environ["LOCALAI_OLLAMA_REGISTRY"]


def test_resumed_download(registry, tmp_path):
    host, _, payload, state = registry
    dst = tmp_path / "big.bin"
    (tmp_path / "big.bin.partial").write_bytes(payload[:1000])  # an interrupted earlier attempt
    state["ranges"].clear()
    download_file(f"http://{host}/files/big.bin", str(dst), sha=hashlib.sha256(payload).hexdigest())
    assert dst.read_bytes() == payload and state["ranges"] == ["bytes=1000-"]
    # a partial that already holds everything: 416, then verified and renamed
    (tmp_path / "b2.partial").write_bytes(payload)
    download_file(f"http://{host}/files/big.bin", str(tmp_path / "b2"), sha=hashlib.sha256(payload).hexdigest())
    assert (tmp_path / "b2").read_bytes() == payload


def _apply_layers(staging, layers):
    for data in layers:
        with tarfile.open(fileobj=io.BytesIO(data), mode="r:*") as tf:
            oci._safe_extract(tf, str(staging))


def test_whiteout_cannot_delete_outside_its_own_image(tmp_path):
    """`.wh..` / `.wh...` / a root-level opaque whiteout only touch entries of earlier layers of
    the SAME image (private staging tree); the user's existing models survive the merge."""
    dest = tmp_path / "models"
    dest.mkdir()
    (dest / "user-model.gguf").write_bytes(b"keep me")
    (dest / "sub").mkdir()
    (dest / "sub" / "keep.txt").write_bytes(b"keep")
    staging = dest / ".oci-staging-test"
    staging.mkdir()
    l1 = _tar({"a.gguf": b"A", "dir/b.txt": b"B"})
    l2 = _tar({".wh..": b"", ".wh...": b"", "dir/.wh..": b"", "dir/.wh...": b"", ".wh.": b""})
    _apply_layers(staging, [l1, l2])
    assert (staging / "a.gguf").read_bytes() == b"A" and (staging / "dir" / "b.txt").exists()
    l3 = _tar({".wh..wh..opq": b"", "c.gguf": b"C"})      # opaque at the image root: drops a.gguf, dir/
    _apply_layers(staging, [l3])
    assert sorted(os.listdir(staging)) == ["c.gguf"]
    oci._merge_into(str(staging), str(dest))
    assert (dest / "user-model.gguf").read_bytes() == b"keep me"
    assert (dest / "sub" / "keep.txt").read_bytes() == b"keep"
    assert (dest / "c.gguf").read_bytes() == b"C"
    assert tmp_path.exists() and dest.exists()


def test_whiteout_of_lower_layer_symlink_removes_only_the_link(tmp_path):
    staging = tmp_path / "st"
    staging.mkdir()
    outside = tmp_path / "outside"
    outside.mkdir()
    (outside / "precious").write_bytes(b"x")
    link = tarfile.TarInfo("lnk")
    link.type = tarfile.SYMTYPE
    link.linkname = "a.gguf"
    _apply_layers(staging, [_tar({"a.gguf": b"A"}, extra=[link])])
    assert os.path.islink(staging / "lnk")
    _apply_layers(staging, [_tar({".wh.lnk": b""})])
    assert not os.path.lexists(staging / "lnk") and (staging / "a.gguf").exists()
    assert (outside / "precious").exists()
