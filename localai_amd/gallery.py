"""Model gallery: index fetch, install, delete, and the async job service
(`core/gallery/{gallery,models,request}.go`, `core/services/gallery.go`).

A gallery is a YAML list of GalleryModel entries hosted at a URL (http(s)://, github:, file://).
Installing a model downloads its files (SHA-256 verified), writes prompt templates as
`<name>.tmpl`, writes `<name>.yaml` (config_file merged with overrides, `name` forced), and a
`._gallery_<name>.yaml` record used later by delete.  Jobs run on one background thread.
"""
from __future__ import annotations

import copy
import logging
import os
import queue
import threading
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import yaml

from .config.backend_config import BackendConfig
from .utils.downloader import download_file, read_uri, verify_path

log = logging.getLogger("localai_amd.gallery")


def gallery_file_name(name: str) -> str:
    return f"._gallery_{name}.yaml"


def deep_merge(dst: dict, src: dict) -> dict:
    """mergo.Merge(..., WithOverride): src wins, maps merged recursively."""
    for k, v in (src or {}).items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            deep_merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


@dataclass
class GalleryModel:
    name: str = ""
    url: str = ""
    description: str = ""
    license: str = ""
    urls: List[str] = field(default_factory=list)
    icon: str = ""
    tags: List[str] = field(default_factory=list)
    config_file: Dict[str, Any] = field(default_factory=dict)
    overrides: Dict[str, Any] = field(default_factory=dict)
    files: List[dict] = field(default_factory=list)
    gallery: Dict[str, str] = field(default_factory=dict)
    installed: bool = False

    @staticmethod
    def from_dict(d: dict) -> "GalleryModel":
        return GalleryModel(name=str(d.get("name") or ""), url=str(d.get("url") or ""),
                            description=str(d.get("description") or ""), license=str(d.get("license") or ""),
                            urls=list(d.get("urls") or []), icon=str(d.get("icon") or ""),
                            tags=list(d.get("tags") or []), config_file=dict(d.get("config_file") or {}),
                            overrides=dict(d.get("overrides") or {}), files=list(d.get("files") or []),
                            gallery=dict(d.get("gallery") or {}))

    def id(self) -> str:
        return f"{self.gallery.get('name', '')}@{self.name}"

    def to_json(self) -> dict:
        d = {"url": self.url, "name": self.name, "description": self.description, "license": self.license,
             "urls": self.urls, "icon": self.icon, "tags": self.tags, "config_file": self.config_file or None,
             "overrides": self.overrides or None, "files": self.files or None, "gallery": self.gallery,
             "installed": self.installed}
        return {k: v for k, v in d.items() if v not in (None, "", [], False) or k in ("name", "gallery")}


def _load_yaml(data: bytes):
    return yaml.safe_load(data.decode("utf-8")) if data else None


def get_gallery_config(url: str, base_path: str) -> dict:
    cfg = _load_yaml(read_uri(url, base_path)) or {}
    if not isinstance(cfg, dict):
        raise ValueError(f"invalid gallery config at {url}")
    return cfg


def gallery_models(gallery: dict, base_path: str) -> List[GalleryModel]:
    url = gallery.get("url", "")
    if url.endswith(".ref"):
        ref = read_uri(url, base_path).decode().strip()
        if not ref:
            raise ValueError(f"invalid reference file at url {url}")
        url = url[:url.rfind("/") + 1] + ref
    items = _load_yaml(read_uri(url, base_path)) or []
    out = []
    for d in items:
        if not isinstance(d, dict):
            continue
        m = GalleryModel.from_dict(d)
        m.gallery = dict(gallery)
        m.installed = os.path.exists(os.path.join(base_path, f"{m.name}.yaml"))
        out.append(m)
    return out


def available_models(galleries: List[dict], base_path: str) -> List[GalleryModel]:
    out: List[GalleryModel] = []
    for g in galleries:
        out += gallery_models(g, base_path)
    return out


def find_model(models: List[GalleryModel], name: str) -> Optional[GalleryModel]:
    name = name.replace(os.sep, "__")
    if "@" not in name:
        for m in models:
            if m.name.lower() == name.lower():
                return m
        return None
    for m in models:
        if name.lower() == m.id().lower():
            return m
    return None


def install_model(base_path: str, name_override: str, config: dict, overrides: Optional[dict],
                  progress: Optional[Callable] = None):
    """InstallModel (core/gallery/models.go:99-217)."""
    os.makedirs(base_path, exist_ok=True)
    files = list(config.get("files") or [])
    for i, f in enumerate(files):
        fn = f.get("filename", "")
        verify_path(fn, base_path)
        download_file(f.get("uri", ""), os.path.join(base_path, fn), f.get("sha256", ""),
                      (lambda n, done, tot, _i=i: progress(n, done, tot, _i, len(files))) if progress else None)
    for t in config.get("prompt_templates") or []:
        verify_path(t["name"] + ".tmpl", base_path)
        p = os.path.join(base_path, t["name"] + ".tmpl")
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as fh:
            fh.write(t.get("content", ""))
    name = name_override or config.get("name", "")
    verify_path(name + ".yaml", base_path)
    if overrides or config.get("config_file"):
        cm = yaml.safe_load(config.get("config_file") or "") or {}
        cm["name"] = name
        deep_merge(cm, overrides or {})
        if not BackendConfig(copy.deepcopy(cm)).validate():
            raise ValueError("failed to validate updated config YAML")
        with open(os.path.join(base_path, name + ".yaml"), "w") as fh:
            yaml.safe_dump(cm, fh, sort_keys=False)
    with open(os.path.join(base_path, gallery_file_name(name)), "w") as fh:
        yaml.safe_dump(config, fh, sort_keys=False)


def install_from_gallery(galleries: List[dict], name: str, base_path: str, req: GalleryModel,
                         progress: Optional[Callable] = None):
    name = name.replace(os.sep, "__")
    model = find_model(available_models(galleries, base_path), name)
    if model is None:
        raise ValueError(f"no model found with name {name!r}")
    if model.url:
        config = get_gallery_config(model.url, base_path)
    elif model.config_file:
        config = {"config_file": yaml.safe_dump(model.config_file), "description": model.description,
                  "license": model.license, "urls": list(model.urls), "name": model.name, "files": []}
    else:
        raise ValueError(f"invalid gallery model {model.name}")
    config["urls"] = list(config.get("urls") or []) + list(model.urls)
    config["icon"] = model.icon
    config["files"] = list(config.get("files") or []) + list(req.files) + list(model.files)
    overrides = deep_merge(copy.deepcopy(model.overrides), req.overrides)
    install_model(base_path, req.name or model.name, config, overrides, progress)


def delete_model(base_path: str, name: str, additional_files: List[str] = ()):
    name = name.replace(os.sep, "__")
    cfg_file = os.path.join(base_path, f"{name}.yaml")
    gal_file = os.path.join(base_path, gallery_file_name(name))
    for f in (f"{name}.yaml", gallery_file_name(name)):
        verify_path(f, base_path)
    to_remove = []
    try:
        with open(gal_file) as fh:
            gc = yaml.safe_load(fh) or {}
        to_remove += [os.path.join(base_path, f["filename"]) for f in gc.get("files") or []]
    except OSError:
        log.error("failed to read gallery file %s", gal_file)
    to_remove += [os.path.join(base_path, f) for f in additional_files]
    to_remove += [cfg_file, gal_file]
    errs = []
    for f in dict.fromkeys(to_remove):
        try:
            os.remove(f)
        except OSError as e:
            errs.append(f"failed to remove file {f}: {e}")
    if errs:
        raise OSError("; ".join(errs))


@dataclass
class GalleryOp:
    id: str
    gallery_model_name: str = ""
    config_url: str = ""
    delete: bool = False
    req: GalleryModel = field(default_factory=GalleryModel)
    galleries: List[dict] = field(default_factory=list)


class GalleryService:
    """services.GalleryService: one worker thread consuming install/delete ops."""

    def __init__(self, app_config, on_change: Optional[Callable[[], None]] = None):
        self.cfg = app_config
        self.on_change = on_change
        self.q: "queue.Queue[GalleryOp]" = queue.Queue()
        self.status: Dict[str, dict] = {}
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._run, daemon=True, name="gallery")
        self._t.start()

    def submit(self, op: GalleryOp) -> str:
        self.update(op.id, {"message": "waiting", "progress": 0, "processed": False})
        self.q.put(op)
        return op.id

    def update(self, uid: str, st: dict):
        with self._lock:
            self.status[uid] = dict(st)

    def get(self, uid: str) -> Optional[dict]:
        with self._lock:
            return self.status.get(uid)

    def all(self) -> Dict[str, dict]:
        with self._lock:
            return dict(self.status)

    def _run(self):
        while True:
            op = self.q.get()
            base = self.cfg.models_path
            self.update(op.id, {"message": "processing", "progress": 0, "processed": False,
                                "deletion": op.delete, "gallery_model_name": op.gallery_model_name})

            def progress(fname, done, total, i=0, n=1):
                pct = (done / total * 100.0) if total else 0.0
                self.update(op.id, {"message": "processing", "file_name": fname, "progress": pct,
                                    "downloaded_size": str(done), "file_size": str(total), "processed": False,
                                    "gallery_model_name": op.gallery_model_name})
            try:
                if op.delete:
                    delete_model(base, op.gallery_model_name)
                elif op.config_url:
                    config = get_gallery_config(op.config_url, base)
                    config["files"] = list(config.get("files") or []) + list(op.req.files)
                    install_model(base, op.req.name, config, op.req.overrides, progress)
                else:
                    install_from_gallery(op.galleries, op.gallery_model_name, base, op.req, progress)
                if self.on_change:
                    self.on_change()
                self.update(op.id, {"processed": True, "message": "completed", "progress": 100,
                                    "deletion": op.delete, "gallery_model_name": op.gallery_model_name})
            except Exception as e:  # job failure is reported through the status
                log.error("gallery op %s failed: %s", op.id, e)
                self.update(op.id, {"error": str(e), "processed": True, "message": "error: " + str(e),
                                    "deletion": op.delete, "gallery_model_name": op.gallery_model_name})


def new_op_id() -> str:
    return str(uuid.uuid4())


def safety_scan_gallery_models(galleries: List[dict], base_path: str, fetch=None) -> List[dict]:
    """core/gallery/gallery.go:242-264: scan the files of every INSTALLED gallery model with the
    Hub's safety scan; returns one {model, uri, clamAV, pickles} record per flagged file.  Only an
    unsafe verdict counts -- unreachable scans and non-HF URIs are skipped, as in the reference."""
    from .utils.downloader import UnsafeFilesFound, hf_scan
    flagged = []
    for m in available_models(galleries, base_path):
        if not m.installed:
            continue
        for f in m.files:
            try:
                hf_scan(f.get("uri", ""), fetch=fetch)
            except UnsafeFilesFound as e:
                flagged.append({"model": m.name, "uri": f.get("uri"), "clamAV": e.result["clamAVInfectedFiles"],
                                "pickles": e.result["dangerousPickles"]})
                break  # the reference stops at the first unsafe file of a model
            except Exception:
                continue
    return flagged

