"""ApplicationConfig: the server-wide options (`core/config/application_config.go:14-387`),
populated from the same CLI flags / env vars as `local-ai run` (`core/cli/run.go:19-73`)."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional


def _env(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return v
    return default


def _bool(v) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def parse_duration(s: str) -> float:
    """Go-style duration ('15m', '5m30s', '1h', '10s') -> seconds."""
    if not s:
        return 0.0
    import re
    total = 0.0
    for num, unit in re.findall(r"([\d.]+)(ms|s|m|h)", s):
        total += float(num) * {"ms": 1e-3, "s": 1, "m": 60, "h": 3600}[unit]
    if total == 0 and s.replace(".", "").isdigit():
        total = float(s)
    return total


@dataclass
class ApplicationConfig:
    models_path: str = "models"
    backend_assets_path: str = "/tmp/localai/backend_data"
    image_dir: str = "/tmp/generated/images"
    audio_dir: str = "/tmp/generated/audio"
    upload_dir: str = "/tmp/localai/upload"
    config_dir: str = "/tmp/localai/config"
    dynamic_config_dir: str = "configuration"
    dynamic_config_poll_interval: float = 0.0
    models_config_file: str = ""
    galleries: List[dict] = field(default_factory=list)
    autoload_galleries: bool = False
    remote_library: str = ""
    preload_models: str = ""
    preload_models_from_path: str = ""
    model_urls: List[str] = field(default_factory=list)
    f16: bool = False
    threads: int = 0
    context_size: int = 512
    address: str = ":8080"
    cors: bool = False
    cors_allow_origins: str = ""
    csrf: bool = False
    upload_limit_mb: int = 15
    api_keys: List[str] = field(default_factory=list)
    disable_webui: bool = False
    disable_predownload_scan: bool = False
    opaque_errors: bool = False
    use_subtle_key_comparison: bool = False
    disable_api_key_requirement_for_http_get: bool = False
    http_get_exempted_endpoints: List[str] = field(default_factory=lambda: [
        "^/$", "^/browse/?$", "^/talk/?$", "^/p2p/?$", "^/chat/?$", "^/text2image/?$", "^/tts/?$", "^/static/.*$",
        "^/swagger.*$"])
    p2p: bool = False
    p2p_token: str = ""
    p2p_network_id: str = ""
    parallel_backend_requests: bool = True
    single_active_backend: bool = False
    preload_backend_only: bool = False
    external_grpc_backends: Dict[str, str] = field(default_factory=dict)
    watchdog_idle: bool = False
    watchdog_idle_timeout: float = 15 * 60.0
    watchdog_busy: bool = False
    watchdog_busy_timeout: float = 5 * 60.0
    federated: bool = False
    disable_gallery_endpoint: bool = False
    load_to_memory: List[str] = field(default_factory=list)
    debug: bool = False
    disable_metrics: bool = False
    # MI355X engine knobs
    engine_mode: str = "inprocess"    # inprocess | process
    gpus: List[int] = field(default_factory=list)

    @staticmethod
    def from_env(**overrides) -> "ApplicationConfig":
        c = ApplicationConfig()
        c.models_path = _env("LOCALAI_MODELS_PATH", "MODELS_PATH", default=c.models_path)
        c.backend_assets_path = _env("LOCALAI_BACKEND_ASSETS_PATH", "BACKEND_ASSETS_PATH", default=c.backend_assets_path)
        c.image_dir = _env("LOCALAI_IMAGE_PATH", "IMAGE_PATH", default=c.image_dir)
        c.audio_dir = _env("LOCALAI_AUDIO_PATH", "AUDIO_PATH", default=c.audio_dir)
        c.upload_dir = _env("LOCALAI_UPLOAD_PATH", "UPLOAD_PATH", default=c.upload_dir)
        c.config_dir = _env("LOCALAI_CONFIG_PATH", "CONFIG_PATH", default=c.config_dir)
        c.dynamic_config_dir = _env("LOCALAI_CONFIG_DIR", default=c.dynamic_config_dir)
        c.dynamic_config_poll_interval = parse_duration(_env("LOCALAI_CONFIG_DIR_POLL_INTERVAL", default="") or "")
        c.models_config_file = _env("LOCALAI_MODELS_CONFIG_FILE", "CONFIG_FILE", default="")
        g = _env("LOCALAI_GALLERIES", "GALLERIES", default="")
        if g:
            try:
                c.galleries = json.loads(g)
            except ValueError:
                pass
        c.autoload_galleries = _bool(_env("LOCALAI_AUTOLOAD_GALLERIES", "AUTOLOAD_GALLERIES", default="false"))
        c.remote_library = _env("LOCALAI_REMOTE_LIBRARY", "REMOTE_LIBRARY", default="")
        c.preload_models = _env("LOCALAI_PRELOAD_MODELS", "PRELOAD_MODELS", default="")
        c.preload_models_from_path = _env("LOCALAI_PRELOAD_MODELS_CONFIG", "PRELOAD_MODELS_CONFIG", default="")
        m = _env("LOCALAI_MODELS", "MODELS", default="")
        c.model_urls = [x for x in m.split(",") if x] if m else []
        c.f16 = _bool(_env("LOCALAI_F16", "F16", default="false"))
        c.threads = int(_env("LOCALAI_THREADS", "THREADS", default="0") or 0)
        c.context_size = int(_env("LOCALAI_CONTEXT_SIZE", "CONTEXT_SIZE", default="512") or 512)
        c.address = _env("LOCALAI_ADDRESS", "ADDRESS", default=c.address)
        c.cors = _bool(_env("LOCALAI_CORS", "CORS", default="false"))
        c.cors_allow_origins = _env("LOCALAI_CORS_ALLOW_ORIGINS", "CORS_ALLOW_ORIGINS", default="")
        c.csrf = _bool(_env("LOCALAI_CSRF", default="false"))
        c.upload_limit_mb = int(_env("LOCALAI_UPLOAD_LIMIT", "UPLOAD_LIMIT", default="15"))
        k = _env("LOCALAI_API_KEY", "API_KEY", default="")
        c.api_keys = [x for x in k.split(",") if x] if k else []
        c.disable_webui = _bool(_env("LOCALAI_DISABLE_WEBUI", "DISABLE_WEBUI", default="false"))
        c.disable_predownload_scan = _bool(_env("LOCALAI_DISABLE_PREDOWNLOAD_SCAN", default="false"))
        c.opaque_errors = _bool(_env("LOCALAI_OPAQUE_ERRORS", default="false"))
        c.use_subtle_key_comparison = _bool(_env("LOCALAI_SUBTLE_KEY_COMPARISON", default="false"))
        c.disable_api_key_requirement_for_http_get = _bool(
            _env("LOCALAI_DISABLE_API_KEY_REQUIREMENT_FOR_HTTP_GET", default="false"))
        ex = _env("LOCALAI_HTTP_GET_EXEMPTED_ENDPOINTS", default="")
        if ex:
            c.http_get_exempted_endpoints = ex.split(",")
        c.p2p = _bool(_env("LOCALAI_P2P", "P2P", default="false"))
        c.p2p_token = _env("LOCALAI_P2P_TOKEN", "P2P_TOKEN", "TOKEN", default="")
        c.p2p_network_id = _env("LOCALAI_P2P_NETWORK_ID", "P2P_NETWORK_ID", default="")
        c.parallel_backend_requests = _bool(_env("LOCALAI_PARALLEL_REQUESTS", "PARALLEL_REQUESTS", default="true"))
        c.single_active_backend = _bool(_env("LOCALAI_SINGLE_ACTIVE_BACKEND", "SINGLE_ACTIVE_BACKEND", default="false"))
        c.preload_backend_only = _bool(_env("LOCALAI_PRELOAD_BACKEND_ONLY", "PRELOAD_BACKEND_ONLY", default="false"))
        eb = _env("LOCALAI_EXTERNAL_GRPC_BACKENDS", "EXTERNAL_GRPC_BACKENDS", default="")
        for item in (eb.split(",") if eb else []):
            name, _, uri = item.partition(":")
            if name and uri:
                c.external_grpc_backends[name] = uri
        c.watchdog_idle = _bool(_env("LOCALAI_WATCHDOG_IDLE", "WATCHDOG_IDLE", default="false"))
        c.watchdog_idle_timeout = parse_duration(_env("LOCALAI_WATCHDOG_IDLE_TIMEOUT", "WATCHDOG_IDLE_TIMEOUT",
                                                      default="15m"))
        c.watchdog_busy = _bool(_env("LOCALAI_WATCHDOG_BUSY", "WATCHDOG_BUSY", default="false"))
        c.watchdog_busy_timeout = parse_duration(_env("LOCALAI_WATCHDOG_BUSY_TIMEOUT", "WATCHDOG_BUSY_TIMEOUT",
                                                      default="5m"))
        c.federated = _bool(_env("LOCALAI_FEDERATED", "FEDERATED", default="false"))
        c.disable_gallery_endpoint = _bool(_env("LOCALAI_DISABLE_GALLERY_ENDPOINT", "DISABLE_GALLERY_ENDPOINT",
                                                default="false"))
        lm = _env("LOCALAI_LOAD_TO_MEMORY", "LOAD_TO_MEMORY", default="")
        c.load_to_memory = [x for x in lm.split(",") if x] if lm else []
        c.debug = _bool(_env("LOCALAI_DEBUG", "DEBUG", default="false"))
        c.engine_mode = _env("LOCALAI_ENGINE_MODE", default=c.engine_mode)
        for k2, v in overrides.items():
            setattr(c, k2, v)
        return c
