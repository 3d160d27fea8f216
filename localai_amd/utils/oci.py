"""OCI registry pulls for `oci://` and `ollama://` model URIs.

Reference: `pkg/oci/image.go` (GetImage + ExtractOCIImage: pull an image for this platform and
unpack its layers into the model directory), `pkg/oci/blob.go` (FetchImageBlob by digest),
`pkg/oci/ollama.go` (registry.ollama.ai manifest -> the `application/vnd.ollama.image.model`
layer -> blob), `pkg/downloader/uri.go:209-233` (dispatch).  The reference's ParseImageParts
tests `strings.Contains("/", image)` (arguments swapped), so `ollama://ns/model:tag` never uses the
namespace; here the namespace is honoured (keep behaviour, not bugs).

Plain OCI distribution API over HTTP(S): manifests negotiated with the OCI / Docker media types,
image indexes resolved to linux/amd64, anonymous bearer tokens obtained from the registry's
`WWW-Authenticate` challenge, blobs streamed to disk and checked against their sha256 digest,
layers (tar, optionally gzip) unpacked with path-traversal and link checks and whiteout handling.
Registries on localhost / 127.0.0.1 or listed in LOCALAI_INSECURE_REGISTRIES use plain http.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import shutil
import tarfile
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, Dict, Optional, Tuple

MANIFEST_TYPES = ", ".join([
    "application/vnd.oci.image.manifest.v1+json", "application/vnd.docker.distribution.manifest.v2+json",
    "application/vnd.oci.image.index.v1+json", "application/vnd.docker.distribution.manifest.list.v2+json"])
INDEX_TYPES = ("application/vnd.oci.image.index.v1+json", "application/vnd.docker.distribution.manifest.list.v2+json")
OLLAMA_MODEL = "application/vnd.ollama.image.model"
DOCKER_HUB = "registry-1.docker.io"


def parse_reference(ref: str, default_registry: str = DOCKER_HUB) -> Tuple[str, str, str]:
    """"[registry/]repo[:tag|@digest]" -> (registry, repository, tag or digest).  A first path
    component with a dot, a colon or "localhost" is a registry host; Docker Hub single names get
    the "library/" namespace."""
    digest = ""
    if "@" in ref:
        ref, digest = ref.split("@", 1)
    parts = ref.split("/")
    if len(parts) > 1 and ("." in parts[0] or ":" in parts[0] or parts[0] == "localhost"):
        registry, rest = parts[0], "/".join(parts[1:])
    else:
        registry, rest = default_registry, ref
    tag = "latest"
    last = rest.rsplit("/", 1)[-1]
    if ":" in last:
        rest, tag = rest.rsplit(":", 1)
    if registry in (DOCKER_HUB, "docker.io", "index.docker.io"):
        registry = DOCKER_HUB
        if "/" not in rest:
            rest = "library/" + rest
    return registry, rest, digest or tag


class Registry:
    def __init__(self, host: str):
        self.host = host
        insecure = {h.strip() for h in os.environ.get("LOCALAI_INSECURE_REGISTRIES", "").split(",") if h.strip()}
        name = host.split(":")[0]
        self.base = f"{'http' if name in ('localhost', '127.0.0.1') or host in insecure else 'https'}://{host}/v2/"
        self._token: Dict[str, str] = {}

    def _auth(self, challenge: str, repo: str) -> Optional[str]:
        m = re.match(r"\s*Bearer\s+(.*)", challenge or "", re.I)
        if not m:
            return None
        params = dict(re.findall(r'(\w+)="([^"]*)"', m.group(1)))
        realm = params.pop("realm", "")
        if not realm:
            return None
        params.setdefault("scope", f"repository:{repo}:pull")
        with urllib.request.urlopen(realm + "?" + urllib.parse.urlencode(params), timeout=60) as r:  # noqa: S310
            doc = json.loads(r.read())
        return doc.get("token") or doc.get("access_token")

    def _open(self, path: str, repo: str, headers: Optional[dict] = None):
        hdr = dict(headers or {})
        if repo in self._token:
            hdr["Authorization"] = "Bearer " + self._token[repo]
        req = urllib.request.Request(self.base + path, headers=hdr)
        try:
            return urllib.request.urlopen(req, timeout=120)  # noqa: S310
        except urllib.error.HTTPError as e:
            if e.code != 401 or repo in self._token:
                raise
            tok = self._auth(e.headers.get("WWW-Authenticate", ""), repo)
            if not tok:
                raise
            self._token[repo] = tok
            hdr["Authorization"] = "Bearer " + tok
            return urllib.request.urlopen(urllib.request.Request(self.base + path, headers=hdr), timeout=120)  # noqa: S310

    def manifest(self, repo: str, ref: str, platform: Tuple[str, str] = ("linux", "amd64")) -> dict:
        with self._open(f"{repo}/manifests/{ref}", repo, {"Accept": MANIFEST_TYPES}) as r:
            doc = json.loads(r.read())
            mt = doc.get("mediaType") or r.headers.get("Content-Type", "")
        if mt in INDEX_TYPES or "manifests" in doc:
            for m in doc.get("manifests", []):
                p = m.get("platform") or {}
                if (p.get("os"), p.get("architecture")) == platform:
                    return self.manifest(repo, m["digest"], platform)
            raise ValueError(f"{self.host}/{repo}:{ref}: no {platform[0]}/{platform[1]} manifest in the index")
        return doc

    def fetch_blob(self, repo: str, digest: str, dst: str,
                   progress: Optional[Callable[[str, int, int], None]] = None, size: int = 0) -> str:
        algo, _, want = digest.partition(":")
        h = hashlib.new(algo or "sha256")
        done = 0
        with self._open(f"{repo}/blobs/{digest}", repo) as r, open(dst, "wb") as f:
            total = size or int(r.headers.get("Content-Length") or 0)
            while True:
                b = r.read(1 << 22)
                if not b:
                    break
                f.write(b)
                h.update(b)
                done += len(b)
                if progress:
                    progress(os.path.basename(dst), done, total)
        if want and h.hexdigest() != want:
            os.remove(dst)
            raise ValueError(f"blob {digest}: digest mismatch ({h.hexdigest()})")
        return dst


def _rm(p: str) -> None:
    if os.path.isdir(p) and not os.path.islink(p):
        shutil.rmtree(p)
    elif os.path.lexists(p):
        os.remove(p)


def _inside(root: str, p: str) -> bool:
    return p.startswith(root + os.sep)


def _safe_extract(tf: tarfile.TarFile, dest: str) -> None:
    """Apply one layer to the image's private staging tree `dest`.  Whiteouts (`.wh.<name>`,
    `.wh..wh..opq`) only ever delete entries of EARLIER LAYERS OF THIS IMAGE, because the staging
    tree holds nothing else; a whiteout whose victim is empty, '.', '..', contains a separator or
    resolves outside (or to) the staging root is ignored."""
    root = os.path.realpath(dest)
    for m in tf.getmembers():
        name = m.name.lstrip("/")
        target = os.path.realpath(os.path.join(root, name))
        if target != root and not _inside(root, target):
            continue  # path traversal
        base = os.path.basename(name)
        if base.startswith(".wh."):  # whiteout: the layer deletes a path of a lower layer
            parent = os.path.realpath(os.path.dirname(os.path.join(root, name)))
            if parent != root and not _inside(root, parent):
                continue
            if base == ".wh..wh..opq":
                if os.path.isdir(parent) and not os.path.islink(parent):
                    for e in os.listdir(parent):
                        _rm(os.path.join(parent, e))
                continue
            vname = base[4:]
            if vname in ("", ".", "..") or "/" in vname or os.sep in vname or vname.startswith(".wh."):
                continue
            victim = os.path.join(parent, vname)
            if not _inside(root, os.path.realpath(victim)) and not _inside(root, os.path.abspath(victim)):
                continue
            if os.path.dirname(os.path.abspath(victim)) != parent:
                continue
            _rm(victim)
            continue
        if m.isdir():
            os.makedirs(target, exist_ok=True)
        elif m.isfile():
            os.makedirs(os.path.dirname(target), exist_ok=True)
            src = tf.extractfile(m)
            if os.path.lexists(target) and (os.path.islink(target) or os.path.isdir(target)):
                _rm(target)
            with open(target, "wb") as out:
                shutil.copyfileobj(src, out)
            os.chmod(target, m.mode & 0o755 | 0o600)
        elif m.issym():
            link = os.path.realpath(os.path.join(os.path.dirname(target), m.linkname))
            if _inside(root, link):
                os.makedirs(os.path.dirname(target), exist_ok=True)
                if os.path.lexists(target):
                    _rm(target)
                os.symlink(m.linkname, target)
        # hard links, devices, fifos: skipped


def _merge_into(staging: str, dest: str) -> None:
    """Move the flattened image into `dest`: files of the image replace same-named files, and
    nothing that was already in `dest` is ever deleted (the reference's mutate.Extract +
    archive.Apply behaviour)."""
    for dirpath, dirnames, filenames in os.walk(staging):
        rel = os.path.relpath(dirpath, staging)
        out_dir = dest if rel == "." else os.path.join(dest, rel)
        if os.path.lexists(out_dir) and not os.path.isdir(out_dir):
            os.remove(out_dir)
        os.makedirs(out_dir, exist_ok=True)
        for d in list(dirnames):
            sp = os.path.join(dirpath, d)
            if os.path.islink(sp):  # symlinked dirs move as links, not walked
                dirnames.remove(d)
                filenames.append(d)
        for f in filenames:
            sp, dp = os.path.join(dirpath, f), os.path.join(out_dir, f)
            if os.path.lexists(dp) and (os.path.isdir(dp) and not os.path.islink(dp)):
                continue  # never replace a directory the user already has
            if os.path.lexists(dp):
                os.remove(dp)
            os.replace(sp, dp)


def pull_image(ref: str, dest: str, progress: Optional[Callable[[str, int, int], None]] = None) -> str:
    """`oci://` model URIs: flatten every layer of the image (linux/amd64) in order in a private
    staging tree, then move the result into `dest`."""
    registry, repo, tag = parse_reference(ref)
    reg = Registry(registry)
    man = reg.manifest(repo, tag)
    os.makedirs(dest, exist_ok=True)
    staging = os.path.join(dest, f".oci-staging-{os.getpid()}")
    if os.path.lexists(staging):
        _rm(staging)
    os.makedirs(staging)
    try:
        for i, layer in enumerate(man.get("layers", [])):
            tmp = os.path.join(dest, f".layer{i}.partial")
            reg.fetch_blob(repo, layer["digest"], tmp, progress, int(layer.get("size") or 0))
            try:
                with tarfile.open(tmp, mode="r:*") as tf:  # plain or gzip tar, random access from disk
                    _safe_extract(tf, staging)
            finally:
                if os.path.exists(tmp):
                    os.remove(tmp)
        _merge_into(staging, dest)
    finally:
        if os.path.lexists(staging):
            _rm(staging)
    return dest


def ollama_fetch_model(ref: str, dst: str, progress: Optional[Callable[[str, int, int], None]] = None,
                       registry: str = "") -> str:
    """`ollama://name[:tag]` or `ollama://ns/name[:tag]`: the model layer of the Ollama manifest."""
    host = registry or os.environ.get("LOCALAI_OLLAMA_REGISTRY", "registry.ollama.ai")
    _, repo, tag = parse_reference(f"{host}/{ref if '/' in ref.split(':')[0] else 'library/' + ref}", host)
    reg = Registry(host)
    man = reg.manifest(repo, tag)
    for layer in man.get("layers", []):
        if layer.get("mediaType") == OLLAMA_MODEL:
            return reg.fetch_blob(repo, layer["digest"], dst, progress, int(layer.get("size") or 0))
    raise ValueError(f"ollama://{ref}: the manifest has no {OLLAMA_MODEL} layer")
