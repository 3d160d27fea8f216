"""Application startup (`core/startup/startup.go`, `pkg/startup/model_preload.go`,
`core/startup/config_file_watcher.go`).

Order: create dirs -> install `--models` (URLs, gallery names, local YAML files) -> load model
configs from the models path and `--models-config-file` -> preload (download) config assets
-> JSON gallery preloads -> dynamic config watcher (api_keys.json, external_backends.json) ->
watchdog -> `load_to_memory` models are loaded eagerly.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os
import threading
from typing import List

import yaml

from . import gallery as gal
from .config.app_config import ApplicationConfig
from .gateway.state import AppState
from .utils.downloader import download_file, filename_from_url, looks_like_url, verify_path

log = logging.getLogger("localai_amd.startup")


def install_models(galleries: List[dict], models_path: str, models: List[str], library_url: str = "") -> List[str]:
    """InstallModels: remote/embedded library name -> config or URL; URL -> download file; local
    YAML -> copy as <md5>.yaml; else gallery name."""
    from . import library
    errors = []
    lib = {}
    if library_url:
        try:
            lib = library.remote_library_shorteners(library_url, models_path)
        except Exception as e:  # best effort, like the reference
            log.warning("[startup] remote library %s: %s", library_url, e)
    for url in models:
        try:
            url = library.model_short_url(lib.get(url) or url)
            if library.exists_in_library(url):
                name = hashlib.md5(url.encode()).hexdigest()
                with open(os.path.join(models_path, name + ".yaml"), "wb") as f:
                    f.write(library.resolve_content(url))
            elif url.startswith(("oci://", "ollama://")):
                # model_preload.go:57-78: the image name becomes the file name ("/" and ":" -> "__")
                name = url.split("://", 1)[1].replace("/", "__").replace(":", "__")
                verify_path(name, models_path)
                dst = os.path.join(models_path, name)
                if not os.path.exists(dst):
                    download_file(url, dst)
                log.info("[startup] installed model from OCI repository: %s", name)
            elif looks_like_url(url):
                fn = filename_from_url(url)
                verify_path(fn, models_path)
                dst = os.path.join(models_path, fn)
                if not os.path.exists(dst):
                    download_file(url, dst)
            elif os.path.exists(url):
                with open(url, "rb") as f:
                    data = f.read()
                name = hashlib.md5(url.encode()).hexdigest()
                with open(os.path.join(models_path, name + ".yaml"), "wb") as f:
                    f.write(data)
            else:
                models_av = gal.available_models(galleries, models_path) if galleries else []
                if gal.find_model(models_av, url) is None:
                    raise ValueError(f"failed resolving model '{url}'")
                gal.install_from_gallery(galleries, url, models_path, gal.GalleryModel())
        except Exception as e:  # keep going, report all
            log.error("[startup] failed installing model %r: %s", url, e)
            errors.append(f"{url}: {e}")
    return errors


def apply_gallery_json(models_path: str, text: str, galleries: List[dict]):
    """ApplyGalleryFromString: a JSON list of gallery requests ({id|url, name, overrides, files})."""
    for item in json.loads(text) or []:
        req = gal.GalleryModel.from_dict(item)
        if item.get("id"):
            gal.install_from_gallery(galleries, item["id"], models_path, req)
        elif item.get("url") or item.get("config_url"):
            cfg = gal.get_gallery_config(item.get("config_url") or item["url"], models_path)
            cfg["files"] = list(cfg.get("files") or []) + list(req.files)
            gal.install_model(models_path, req.name, cfg, req.overrides)


class ConfigWatcher:
    """Dynamic config dir: api_keys.json replaces/extends the API keys, external_backends.json
    adds external gRPC backends.  Polls mtimes (fsnotify is not available here)."""

    def __init__(self, app: ApplicationConfig, interval: float = 2.0):
        self.app = app
        self.interval = app.dynamic_config_poll_interval or interval
        self.base_keys = list(app.api_keys)
        self.base_ext = dict(app.external_grpc_backends)
        self._mtimes = {}
        self._stop = threading.Event()
        self.handlers = {"api_keys.json": self._api_keys, "external_backends.json": self._external}
        for f in self.handlers:
            self._call(f)

    def _call(self, name):
        p = os.path.join(self.app.dynamic_config_dir, name)
        try:
            with open(p, "rb") as f:
                content = f.read()
        except FileNotFoundError:
            content = b""
        except OSError as e:
            log.error("could not read %s: %s", p, e)
            return
        try:
            self.handlers[name](content)
        except Exception as e:
            log.error("dynamic config %s failed: %s", name, e)

    def _api_keys(self, content: bytes):
        keys = json.loads(content) if content else []
        self.app.api_keys = self.base_keys + [k for k in keys if isinstance(k, str)]

    def _external(self, content: bytes):
        ext = json.loads(content) if content else {}
        self.app.external_grpc_backends = {**self.base_ext, **{str(k): str(v) for k, v in ext.items()}}

    def poll_once(self):
        for name in self.handlers:
            p = os.path.join(self.app.dynamic_config_dir, name)
            try:
                m = os.stat(p).st_mtime_ns
            except OSError:
                m = None
            if self._mtimes.get(name) != m:
                self._mtimes[name] = m
                self._call(name)

    def start(self):
        def run():
            while not self._stop.wait(self.interval):
                self.poll_once()
        threading.Thread(target=run, daemon=True, name="config-watcher").start()

    def stop(self):
        self._stop.set()


def startup(app: ApplicationConfig) -> AppState:
    for d in (app.models_path, app.image_dir, app.audio_dir, app.upload_dir):
        if d:
            os.makedirs(d, exist_ok=True)
    if app.model_urls:
        install_models(app.galleries, app.models_path, app.model_urls, app.remote_library)
    state = AppState(app)
    lo = state.load_options()
    state.configs.load_from_path(app.models_path, lo)
    if app.models_config_file:
        state.configs.load_multiple_single_file(app.models_config_file, lo)
    try:
        state.configs.preload(app.models_path)
    except Exception as e:
        log.error("error downloading models: %s", e)
    if app.preload_models:
        apply_gallery_json(app.models_path, app.preload_models, app.galleries)
    if app.preload_models_from_path:
        with open(app.preload_models_from_path) as f:
            apply_gallery_json(app.models_path, json.dumps(yaml.safe_load(f)), app.galleries)
    if app.dynamic_config_dir:
        os.makedirs(app.dynamic_config_dir, exist_ok=True)
        state.watcher = ConfigWatcher(app)
        state.watcher.start()
    return state


async def load_to_memory(state: AppState):
    for name in state.cfg.load_to_memory:
        cfg = state.config_for(name)
        log.info("preloading %s into memory", name)
        await state.manager.load(cfg)


def run_server(state: AppState, host: str, port: int, server: str = "native"):
    from .gateway.app import create_app
    app = create_app(state)

    async def main():
        if state.cfg.load_to_memory:
            await load_to_memory(state)
        if server == "uvicorn":
            import uvicorn
            srv = uvicorn.Server(uvicorn.Config(app, host=host, port=port, log_level="info"))
            await srv.serve()
        else:
            from .gateway.native_server import NativeHTTPServer
            srv = NativeHTTPServer(app, host, port)
            log.info("LocalAI (MI355X) API listening on %s:%d", host, srv.port)
            await srv.serve()
    asyncio.run(main())
