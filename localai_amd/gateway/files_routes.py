"""OpenAI Files + Assistants API (`core/http/endpoints/openai/{files,assistant}.go`).

State is persisted as JSON in the config dir (`uploadedFiles.json`, `assistants.json`,
`assistantsFile.json`) like the reference's utils.SaveConfig/LoadConfig; uploads go to the upload
dir.  Guarded by one lock (the reference mutates global slices without one)."""
from __future__ import annotations

import json
import os
import random
import threading
import time
from typing import List

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, PlainTextResponse, Response

from ..utils.downloader import sanitize_file_name
from ..utils.multipart import read_form

FILES_JSON = "uploadedFiles.json"
ASSISTANTS_JSON = "assistants.json"
ASSISTANT_FILES_JSON = "assistantsFile.json"
MAX_FILE_IDS = 20


class _Store:
    def __init__(self, cfg):
        self.cfg = cfg
        self.lock = threading.Lock()
        self.files: List[dict] = self._load(FILES_JSON)
        self.assistants: List[dict] = self._load(ASSISTANTS_JSON)
        self.assistant_files: List[dict] = self._load(ASSISTANT_FILES_JSON)
        self.next_file = 1 + max([int(f["id"].split("-")[-1]) for f in self.files
                                  if f.get("id", "").split("-")[-1].isdigit()] or [0])

    def _path(self, name):
        return os.path.join(self.cfg.config_dir, name)

    def _load(self, name) -> list:
        try:
            with open(self._path(name)) as f:
                v = json.load(f)
                return v if isinstance(v, list) else []
        except (OSError, ValueError):
            return []

    def save(self, name, data):
        try:
            os.makedirs(self.cfg.config_dir, exist_ok=True)
            tmp = self._path(name) + ".tmp"
            with open(tmp, "w") as f:
                json.dump(data, f, indent=2)
            os.replace(tmp, self._path(name))
        except OSError:
            pass


def _err(code, msg):
    return PlainTextResponse(msg, status_code=code)


def build_router(state) -> APIRouter:
    r = APIRouter()
    st = _Store(state.cfg)
    state.files = st

    def both(path, fn, method):
        r.add_api_route("/v1" + path, fn, methods=[method])
        r.add_api_route(path, fn, methods=[method])

    # ------------------------------------------------------------------ files
    async def upload(request: Request):
        form = await read_form(request)
        up = form.get("file")
        if up is None:
            return _err(400, "file is required")
        data = await up.read()
        limit = state.cfg.upload_limit_mb * 1024 * 1024
        if len(data) > limit:
            return _err(400, f"File size {len(data)} exceeds upload limit {state.cfg.upload_limit_mb}")
        purpose = form.get("purpose") or ""
        if not purpose:
            return _err(400, "Purpose is not defined")
        name = sanitize_file_name(up.filename or "upload")
        os.makedirs(state.cfg.upload_dir, exist_ok=True)
        dst = os.path.join(state.cfg.upload_dir, name)
        if os.path.exists(dst):
            return _err(400, "File already exists")
        with open(dst, "wb") as f:
            f.write(data)
        with st.lock:
            fid = st.next_file
            st.next_file += 1
            rec = {"id": f"file-{fid}", "object": "file", "bytes": len(data), "created_at": int(time.time()),
                   "filename": name, "purpose": purpose}
            st.files.append(rec)
            st.save(FILES_JSON, st.files)
        return rec

    async def list_files(request: Request):
        purpose = request.query_params.get("purpose", "")
        with st.lock:
            data = [f for f in st.files if not purpose or f.get("purpose") == purpose]
        return {"data": data, "object": "list"}

    def _find(fid):
        for f in st.files:
            if f["id"] == fid:
                return f
        return None

    async def get_file(file_id: str):
        f = _find(file_id)
        if f is None:
            return _err(500, f"unable to find file id {file_id}")
        return f

    async def delete_file(file_id: str):
        with st.lock:
            f = _find(file_id)
            if f is None:
                return _err(500, f"unable to find file id {file_id}")
            try:
                os.remove(os.path.join(state.cfg.upload_dir, f["filename"]))
            except FileNotFoundError:
                pass
            except OSError as e:
                return _err(500, f"Unable to delete file: {f['filename']}, {e}")
            st.files.remove(f)
            st.save(FILES_JSON, st.files)
        return {"id": file_id, "object": "file", "deleted": True}

    async def file_content(file_id: str):
        f = _find(file_id)
        if f is None:
            return _err(500, f"unable to find file id {file_id}")
        try:
            with open(os.path.join(state.cfg.upload_dir, f["filename"]), "rb") as fh:
                return Response(fh.read())
        except OSError as e:
            return _err(500, str(e))

    both("/files", upload, "POST")
    both("/files", list_files, "GET")
    both("/files/{file_id}", get_file, "GET")
    both("/files/{file_id}", delete_file, "DELETE")
    both("/files/{file_id}/content", file_content, "GET")

    # ------------------------------------------------------------------ assistants
    def model_exists(name: str) -> bool:
        return name in state.list_models()

    async def create_assistant(request: Request):
        try:
            b = await request.json()
        except Exception:
            return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
        model = b.get("model", "")
        if not model_exists(model):
            return _err(400, f"Model {model} not found")
        a = {"id": "asst_" + str(random.randint(1, 2 ** 62)), "object": "assistant", "created": int(time.time()),
             "model": model, "name": b.get("name", ""), "description": b.get("description", ""),
             "instructions": b.get("instructions", ""), "tools": b.get("tools") or [],
             "file_ids": b.get("file_ids") or [], "metadata": b.get("metadata") or {}}
        with st.lock:
            st.assistants.append(a)
            st.save(ASSISTANTS_JSON, st.assistants)
        return a

    def _aid(a):
        try:
            return int(a["id"].removeprefix("asst_"))
        except ValueError:
            return None

    async def list_assistants(request: Request):
        q = request.query_params
        try:
            limit = int(q.get("limit", "20"))
        except ValueError:
            return _err(400, f"Invalid limit query value: {q.get('limit')}")
        order = q.get("order", "desc")
        with st.lock:
            out = sorted(st.assistants, key=lambda a: a["created"], reverse=(order != "asc"))
        for key, cmp in (("after", lambda x, y: x > y), ("before", lambda x, y: x < y)):
            v = q.get(key)
            if v and v.lstrip("-").isdigit():
                out = [a for a in out if _aid(a) is not None and cmp(_aid(a), int(v))]
        return out[:limit] if limit < len(out) else out

    def _get_asst(aid):
        for a in st.assistants:
            if a["id"] == aid:
                return a
        return None

    async def get_assistant(assistant_id: str):
        a = _get_asst(assistant_id)
        if a is None:
            return _err(404, f"Unable to find assistant with id: {assistant_id}")
        return a

    async def delete_assistant(assistant_id: str):
        with st.lock:
            a = _get_asst(assistant_id)
            if a is not None:
                st.assistants.remove(a)
                st.save(ASSISTANTS_JSON, st.assistants)
                return {"id": assistant_id, "object": "assistant.deleted", "deleted": True}
        return JSONResponse({"id": assistant_id, "object": "assistant.deleted", "deleted": False}, status_code=404)

    async def modify_assistant(assistant_id: str, request: Request):
        try:
            b = await request.json()
        except Exception:
            return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
        with st.lock:
            a = _get_asst(assistant_id)
            if a is None:
                return _err(404, f"Unable to find assistant with id: {assistant_id}")
            for k in ("model", "name", "description", "instructions", "tools", "file_ids", "metadata"):
                if k in b:
                    a[k] = b[k]
            st.save(ASSISTANTS_JSON, st.assistants)
            return a

    async def create_assistant_file(assistant_id: str, request: Request):
        try:
            b = await request.json()
        except Exception:
            return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
        with st.lock:
            a = _get_asst(assistant_id)
            if a is None:
                return _err(404, f"Unable to find {assistant_id!r}")
            if len(a["file_ids"]) > MAX_FILE_IDS:
                return _err(400, f"Max files {MAX_FILE_IDS} for assistant {a['name']} reached.")
            f = _find(b.get("file_id", ""))
            if f is None:
                return _err(404, f"Unable to find file_id: {b.get('file_id', '')}")
            a["file_ids"].append(f["id"])
            af = {"id": f["id"], "object": "assistant.file", "created_at": int(time.time()), "assistant_id": a["id"]}
            st.assistant_files.append(af)
            st.save(ASSISTANTS_JSON, st.assistants)
            st.save(ASSISTANT_FILES_JSON, st.assistant_files)
            return af

    async def list_assistant_files(assistant_id: str, request: Request):
        q = request.query_params
        try:
            limit = int(q.get("limit", "20"))
        except ValueError:
            limit = 20
        if limit < 1 or limit > 100:
            limit = 20
        with st.lock:
            fs = sorted(st.assistant_files, key=lambda f: f["created_at"], reverse=q.get("order", "desc") != "asc")
        fs = fs[:limit]
        return {"object": "list", "data": fs, "first_id": fs[0]["id"] if fs else "",
                "last_id": fs[-1]["id"] if fs else "", "has_more": False}

    async def delete_assistant_file(assistant_id: str, file_id: str):
        with st.lock:
            a = _get_asst(assistant_id)
            if a is not None and file_id in a["file_ids"]:
                a["file_ids"].remove(file_id)
                st.assistant_files = [f for f in st.assistant_files
                                      if not (f["id"] == file_id and f["assistant_id"] == assistant_id)]
                st.save(ASSISTANTS_JSON, st.assistants)
                st.save(ASSISTANT_FILES_JSON, st.assistant_files)
                return {"id": file_id, "object": "assistant.file.deleted", "deleted": True}
        return JSONResponse({"id": file_id, "object": "assistant.file.deleted", "deleted": False}, status_code=404)

    async def get_assistant_file(assistant_id: str, file_id: str):
        for f in st.assistant_files:
            if f["assistant_id"] == assistant_id:
                if f["id"] == file_id:
                    return f
        if _get_asst(assistant_id) is None:
            return _err(404, f"Unable to find assistant file with assistant_id: {assistant_id}")
        return _err(404, f"Unable to find assistant file with file_id: {file_id}")

    both("/assistants", create_assistant, "POST")
    both("/assistants", list_assistants, "GET")
    both("/assistants/{assistant_id}", get_assistant, "GET")
    both("/assistants/{assistant_id}", modify_assistant, "POST")
    both("/assistants/{assistant_id}", delete_assistant, "DELETE")
    both("/assistants/{assistant_id}/files", create_assistant_file, "POST")
    both("/assistants/{assistant_id}/files", list_assistant_files, "GET")
    both("/assistants/{assistant_id}/files/{file_id}", get_assistant_file, "GET")
    both("/assistants/{assistant_id}/files/{file_id}", delete_assistant_file, "DELETE")
    return r
