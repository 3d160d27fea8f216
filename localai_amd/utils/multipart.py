"""Minimal multipart/form-data parser (python-multipart is not available in this image).
Used by the file-upload and audio-transcription endpoints."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Tuple


@dataclass
class UploadedFile:
    filename: str
    content_type: str
    data: bytes

    async def read(self) -> bytes:
        return self.data


def _params(header_value: str) -> Tuple[str, Dict[str, str]]:
    parts = [p.strip() for p in header_value.split(";")]
    out = {}
    for p in parts[1:]:
        if "=" in p:
            k, v = p.split("=", 1)
            v = v.strip()
            if len(v) >= 2 and v[0] == v[-1] == '"':
                v = v[1:-1]
            out[k.strip().lower()] = v
    return parts[0].lower(), out


def parse_multipart(body: bytes, content_type: str) -> Dict[str, object]:
    """Returns {field_name: str | UploadedFile}."""
    kind, params = _params(content_type)
    if kind != "multipart/form-data" or "boundary" not in params:
        raise ValueError("expected multipart/form-data with a boundary")
    delim = b"--" + params["boundary"].encode("latin-1")
    out: Dict[str, object] = {}
    for chunk in body.split(delim)[1:]:
        if chunk.startswith(b"--"):
            break
        if chunk.startswith(b"\r\n"):
            chunk = chunk[2:]
        head, sep, data = chunk.partition(b"\r\n\r\n")
        if not sep:
            continue
        if data.endswith(b"\r\n"):
            data = data[:-2]
        hdrs = {}
        for line in head.decode("utf-8", "replace").split("\r\n"):
            if ":" in line:
                k, v = line.split(":", 1)
                hdrs[k.strip().lower()] = v.strip()
        _, dp = _params(hdrs.get("content-disposition", ""))
        name = dp.get("name", "")
        if "filename" in dp:
            out[name] = UploadedFile(dp["filename"], hdrs.get("content-type", "application/octet-stream"), data)
        else:
            out[name] = data.decode("utf-8", "replace")
    return out


async def read_form(request) -> Dict[str, object]:
    body = await request.body()
    ct = request.headers.get("content-type", "")
    if ct.startswith("application/x-www-form-urlencoded"):
        from urllib.parse import parse_qsl
        return dict(parse_qsl(body.decode("utf-8", "replace")))
    return parse_multipart(body, ct)
