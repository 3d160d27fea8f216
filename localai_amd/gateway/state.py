"""Server state shared by all routes: configs, model manager, templates, metrics."""
from __future__ import annotations

import os
import time
from typing import List, Optional

from ..config.app_config import ApplicationConfig
from ..config.backend_config import BackendConfig
from ..config.loader import BackendConfigLoader, LoadOptions
from ..templates import TemplateCache
from .metrics import Metrics
from .model_manager import ModelManager

KNOWN_FILES_TO_SKIP = {"model_card", "readme", "readme.md"}
KNOWN_SUFFIX_TO_SKIP = (".tmpl", ".keep", ".yaml", ".yml", ".json", ".txt", ".md", ".MD", ".DS_Store", ".",
                        ".partial", ".tar.gz")
SKIP_IF_CONFIGURED, SKIP_ALWAYS, ALWAYS_INCLUDE, LOOSE_ONLY = range(4)


class AppState:
    def __init__(self, app_config: ApplicationConfig):
        self.cfg = app_config
        self.models_path = app_config.models_path
        os.makedirs(self.models_path, exist_ok=True)
        self.configs = BackendConfigLoader(self.models_path)
        self.manager = ModelManager(app_config, self.models_path)
        self.templates = TemplateCache(self.models_path)
        self.metrics = Metrics()
        self.start_time = time.time()
        self.gallery = None
        self.files = None
        self.assistants = None

    def load_options(self) -> LoadOptions:
        c = self.cfg
        return LoadOptions(model_path=self.models_path, debug=c.debug, threads=c.threads, ctx_size=c.context_size,
                           f16=c.f16)

    def list_files_in_model_path(self) -> List[str]:
        out = []
        try:
            names = sorted(os.listdir(self.models_path))
        except OSError:
            return out
        for n in names:
            if n.lower() in KNOWN_FILES_TO_SKIP or n in KNOWN_FILES_TO_SKIP:
                continue
            if any(n.endswith(s) for s in KNOWN_SUFFIX_TO_SKIP):
                continue
            if os.path.isdir(os.path.join(self.models_path, n)):
                continue
            out.append(n)
        return out

    EXISTS_TTL = 2.0   # seconds a model-path existence answer is reused (one stat per template lookup otherwise)

    def exists_in_model_path(self, name: str) -> bool:
        if not name or "/" in name or ".." in name:
            return False
        cache = self.__dict__.setdefault("_exists_cache", {})
        now = time.monotonic()
        hit = cache.get(name)
        if hit is not None and now - hit[1] < self.EXISTS_TTL:
            return hit[0]
        ok = os.path.exists(os.path.join(self.models_path, name))
        if len(cache) > 4096:
            cache.clear()
        cache[name] = (ok, now)
        return ok

    def list_models(self, flt=None, policy: int = SKIP_IF_CONFIGURED) -> List[str]:
        """services.ListModels (core/services/list_models.go:17-49)."""
        flt = flt or (lambda n, c: True)
        out, skip = [], set()
        if policy != LOOSE_ONLY:
            for c in self.configs.by_filter(flt):
                if policy == SKIP_IF_CONFIGURED:
                    skip.add(c.model)
                out.append(c.name)
        if policy != SKIP_ALWAYS:
            for m in self.list_files_in_model_path():
                if m not in skip and flt(m, None):
                    out.append(m)
        return out

    def config_for(self, model_name: str) -> BackendConfig:
        return self.configs.load_by_name(model_name, self.load_options())
