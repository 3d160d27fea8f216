"""Model/file downloader (`pkg/downloader/uri.go`, `pkg/utils/path.go`).

URI schemes: http(s)://, file://, huggingface://owner/repo/file[@branch], github:org/repo/path[@br],
github://org/repo/path[@br].  Downloads stream to `<dst>.partial`, are SHA-256 checked when a hash
is given, then renamed atomically.  `oci://` images are unpacked into the model directory and
`ollama://` models fetched as their model blob (utils/oci.py).  An interrupted http(s) download
resumes from its `.partial` with a Range request when the server supports it (the reference
deletes the partial and starts over, `pkg/downloader/uri.go:193-205`).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, Optional

HF_PREFIX = "huggingface://"
HF_PREFIX2 = "hf://"
GITHUB = "github:"
GITHUB2 = "github://"
LOCAL = "file://"
OCI = "oci://"
OLLAMA = "ollama://"


def looks_like_url(s: str) -> bool:
    return s.startswith(("http://", "https://", HF_PREFIX, HF_PREFIX2, GITHUB, OCI, OLLAMA))


def resolve_url(s: str) -> str:
    def gh(rest: str) -> str:
        repo, _, branch = rest.partition("@")
        parts = repo.split("/")
        return "https://raw.githubusercontent.com/%s/%s/%s/%s" % (parts[0], parts[1], branch or "main",
                                                                  "/".join(parts[2:]))
    if s.startswith(GITHUB2):
        return gh(s[len(GITHUB2):])
    if s.startswith(GITHUB):
        return gh(s[len(GITHUB):])
    for p in (HF_PREFIX, HF_PREFIX2):
        if s.startswith(p):
            rest = s[len(p):]
            parts = rest.split("/")
            owner, repo = parts[0], parts[1]
            path = "/".join(parts[2:])
            branch = "main"
            if "@" in path:
                path, branch = path.split("@", 1)
            return f"https://huggingface.co/{owner}/{repo}/resolve/{branch}/{path}"
    return s


def filename_from_url(url: str) -> str:
    name = os.path.basename(urllib.parse.urlparse(resolve_url(url)).path)
    if not name:
        raise ValueError(f"cannot derive a file name from {url!r}")
    return name


def verify_path(path: str, base: str):
    """VerifyPath: `base/path` must stay inside base."""
    base_c = os.path.normpath(os.path.abspath(base))
    full = os.path.normpath(os.path.join(base_c, path))
    if full != base_c and not full.startswith(base_c + os.sep):
        raise ValueError("path is outside of trusted root")
    if full == base_c:
        raise ValueError("path is outside of trusted root")


def sanitize_file_name(name: str) -> str:
    return os.path.basename(os.path.normpath(name)).replace("..", "")


def sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def read_uri(uri: str, base_path: str = "") -> bytes:
    """DownloadWithCallback: fetch a (small) resource, file:// restricted to base_path."""
    if uri.startswith(LOCAL):
        p = uri[len(LOCAL):]
        if base_path:
            # like the reference: a file:// resource must resolve (symlinks included) inside base_path
            if not os.path.isabs(p):
                p = os.path.join(base_path, p)
            real, root = os.path.realpath(p), os.path.realpath(base_path)
            if not real.startswith(root + os.sep):
                raise ValueError("path is outside of trusted root")
            p = real
        with open(p, "rb") as f:
            return f.read()
    with urllib.request.urlopen(resolve_url(uri), timeout=60) as r:  # noqa: S310
        return r.read()


def download_file(uri: str, dst: str, sha: str = "",
                  progress: Optional[Callable[[str, int, int], None]] = None, auth: str = ""):
    """DownloadFile: skip if present with matching hash; stream to .partial; verify; rename."""
    if uri.startswith(OCI):  # uri.go:226-232: the image's layers go into the model directory
        from .oci import pull_image
        pull_image(uri[len(OCI):], os.path.dirname(os.path.abspath(dst)) or ".", progress)
        return dst
    if os.path.exists(dst):
        if not sha or sha256_file(dst).lower() == sha.lower():
            return dst
        os.remove(dst)
    os.makedirs(os.path.dirname(os.path.abspath(dst)) or ".", exist_ok=True)
    tmp = dst + ".partial"
    if uri.startswith(LOCAL):
        shutil.copyfile(uri[len(LOCAL):], tmp)
    elif uri.startswith(OLLAMA):
        from .oci import ollama_fetch_model
        ollama_fetch_model(uri[len(OLLAMA):], tmp, progress)
    else:
        req = urllib.request.Request(resolve_url(uri))
        if auth:
            req.add_header("Authorization", auth)
        elif os.environ.get("HUGGINGFACE_HUB_TOKEN") and "huggingface.co" in req.full_url:
            req.add_header("Authorization", "Bearer " + os.environ["HUGGINGFACE_HUB_TOKEN"])
        have = os.path.getsize(tmp) if os.path.exists(tmp) else 0
        if have:  # an earlier attempt left a partial: ask for the rest only
            req.add_header("Range", f"bytes={have}-")
        try:
            r = urllib.request.urlopen(req, timeout=60)  # noqa: S310
        except urllib.error.HTTPError as e:
            if not (e.code == 416 and have):  # 416: the partial already holds the whole file
                raise
            r = None
        if r is not None:
            resumed = bool(have) and r.status == 206
            with r, open(tmp, "ab" if resumed else "wb") as f:
                done = have if resumed else 0
                total = int(r.headers.get("Content-Length") or 0) + done
                while True:
                    b = r.read(1 << 22)
                    if not b:
                        break
                    f.write(b)
                    done += len(b)
                    if progress:
                        progress(os.path.basename(dst), done, total)
    if sha:
        got = sha256_file(tmp)
        if got.lower() != sha.lower():
            os.remove(tmp)
            raise ValueError(f"SHA mismatch for file {dst!r} ( calculated: {got} != metadata: {sha} )")
    os.replace(tmp, dst)
    return dst


# ------------------------------------------------------------------ HuggingFace safety scan
# pkg/downloader/huggingface.go:12-49: ask the Hub's scan API about a repository's files
# (ClamAV + dangerous pickle imports).  Best effort, as in the reference: only huggingface URIs.

class NonHuggingFaceFile(ValueError):
    pass


class UnsafeFilesFound(RuntimeError):
    def __init__(self, result: dict):
        super().__init__("unsafe files found")
        self.result = result


def hf_scan(uri: str, fetch: Optional[Callable[[str], bytes]] = None) -> dict:
    """Returns the scan result ({repositoryId, revision, hasUnsafeFile, clamAVInfectedFiles,
    dangerousPickles, scansDone}); raises UnsafeFilesFound when the Hub flags a file."""
    import json
    parts = resolve_url(uri).split("/")
    if len(parts) <= 4 or parts[2] != "huggingface.co":
        raise NonHuggingFaceFile("not a huggingface repo")
    url = f"https://huggingface.co/api/models/{parts[3]}/{parts[4]}/scan"
    if fetch is None:
        def fetch(u: str) -> bytes:
            with urllib.request.urlopen(u, timeout=30) as r:
                if r.status != 200:
                    raise RuntimeError(f"unexpected status code during HuggingFaceScan: {r.status}")
                return r.read()
    res = json.loads(fetch(url))
    res.setdefault("clamAVInfectedFiles", [])
    res.setdefault("dangerousPickles", [])
    if res.get("hasUnsafeFile"):
        raise UnsafeFilesFound(res)
    return res
