"""BackendConfigLoader (`core/config/backend_config_loader.go:21-358`) and the /v1/models
filters (`core/config/backend_config_filter.go`)."""
from __future__ import annotations

import logging
import os
import re
import threading
from typing import Callable, Dict, List, Optional

from .backend_config import BackendConfig, load_yaml_configs

log = logging.getLogger("localai_amd.config")


class LoadOptions:
    def __init__(self, model_path: str = "", debug: bool = False, threads: int = 0, ctx_size: int = 0,
                 f16: bool = False):
        self.model_path, self.debug, self.threads, self.ctx_size, self.f16 = model_path, debug, threads, ctx_size, f16

    def apply(self, cfg: BackendConfig):
        cfg.set_defaults(ctx=self.ctx_size, threads=self.threads, f16=self.f16, debug=self.debug,
                         model_path=self.model_path)


class BackendConfigLoader:
    def __init__(self, model_path: str):
        self.model_path = model_path
        self.configs: Dict[str, BackendConfig] = {}
        self._lock = threading.RLock()

    def _read_file(self, path: str, lo: LoadOptions) -> List[BackendConfig]:
        with open(path, "r", encoding="utf-8") as f:
            cfgs = load_yaml_configs(f.read())
        for c in cfgs:
            lo.apply(c)
        return cfgs

    def load_backend_config(self, path: str, lo: Optional[LoadOptions] = None):
        lo = lo or LoadOptions(model_path=self.model_path)
        cfgs = self._read_file(path, lo)
        if not cfgs:
            raise ValueError(f"empty config file {path}")
        c = cfgs[0]
        if not c.validate():
            raise ValueError("config is not valid")
        with self._lock:
            self.configs[c.name] = c

    def load_multiple_single_file(self, path: str, lo: Optional[LoadOptions] = None):
        lo = lo or LoadOptions(model_path=self.model_path)
        for c in self._read_file(path, lo):
            if c.validate():
                with self._lock:
                    self.configs[c.name] = c

    def load_from_path(self, path: str, lo: Optional[LoadOptions] = None):
        lo = lo or LoadOptions(model_path=self.model_path)
        if not os.path.isdir(path):
            return
        for fn in sorted(os.listdir(path)):
            if (".yaml" not in fn and ".yml" not in fn) or fn.startswith("."):
                continue
            try:
                cfgs = self._read_file(os.path.join(path, fn), lo)
            except Exception as e:
                log.error("cannot read config file %s: %s", fn, e)
                continue
            for c in cfgs[:1]:
                if c.validate():
                    with self._lock:
                        self.configs[c.name] = c
                else:
                    log.error("config %s is not valid", fn)

    def get(self, name: str) -> Optional[BackendConfig]:
        with self._lock:
            c = self.configs.get(name)
            return c.copy() if c is not None else None

    def add(self, cfg: BackendConfig):
        with self._lock:
            self.configs[cfg.name] = cfg

    def remove(self, name: str):
        with self._lock:
            self.configs.pop(name, None)

    def all(self) -> List[BackendConfig]:
        with self._lock:
            return sorted((c.copy() for c in self.configs.values()), key=lambda c: c.name)

    def by_filter(self, fn: Optional[Callable[[str, BackendConfig], bool]]) -> List[BackendConfig]:
        with self._lock:
            items = list(self.configs.items())
        return [c.copy() for n, c in items if fn is None or fn(n, c)]

    def load_by_name(self, model_name: str, lo: LoadOptions) -> BackendConfig:
        """LoadBackendConfigFileByName: existing config, else `<models>/<name>.yaml`, else defaults."""
        cfg = self.get(model_name)
        if cfg is None:
            p = os.path.join(lo.model_path or self.model_path, model_name + ".yaml")
            if os.path.isfile(p):
                self.load_backend_config(p, lo)
                cfg = self.get(model_name)
        if cfg is None:
            cfg = BackendConfig({"parameters": {"model": model_name}})
        lo.apply(cfg)
        return cfg

    def preload(self, model_path: str, progress=None):
        """Download `download_files` / URL models / mmproj (with SHA-256 verification)."""
        from ..utils.downloader import download_file, verify_path
        with self._lock:
            items = list(self.configs.items())
        for name, cfg in items:
            for f in cfg.raw.get("download_files") or []:
                fn = f.get("filename", "")
                verify_path(fn, model_path)
                download_file(f.get("uri", ""), os.path.join(model_path, fn), f.get("sha256", ""), progress)
            if cfg.is_model_url():
                fn = cfg.model_file_name()
                dst = os.path.join(model_path, fn)
                if not os.path.exists(dst):
                    download_file(cfg.model, dst, "", progress)
                cfg.model = fn
            mm = str(cfg.raw.get("mmproj") or "")
            if mm and cfg.mmproj_file_name() != mm:
                fn = cfg.mmproj_file_name()
                dst = os.path.join(model_path, fn)
                if not os.path.exists(dst):
                    download_file(mm, dst, "", progress)
                cfg.raw["mmproj"] = fn


def build_name_filter(pattern: str) -> Callable[[str, BackendConfig], bool]:
    if not pattern:
        return lambda n, c: True
    rx = re.compile(pattern)
    return lambda n, c: bool(rx.search(n))


def build_usecase_filter(flags: int) -> Callable[[str, BackendConfig], bool]:
    return lambda n, c: c.has_usecases(flags)
