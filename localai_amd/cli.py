"""`local-ai`-compatible command line (`main.go`, `core/cli/*`).

    python -m localai_amd run [MODEL_URLS...] [--models-path DIR] [--address :8080] ...
    python -m localai_amd models list|install NAME
    python -m localai_amd tts TEXT --model M [--backend B] [--voice V] [--output-file F]
    python -m localai_amd sound-generation TEXT --model M ...
    python -m localai_amd transcript FILE --model M [--language L]
    python -m localai_amd util gguf-info FILE | usecase-heuristic FILE
    python -m localai_amd worker tp --model FILE ...   (tensor-parallel worker group, RCCL)

Every `run` flag mirrors the reference flag name and its LOCALAI_* / legacy env variable
(core/cli/run.go:19-73); flags win over env, env over defaults.  `.env` / `localai.env`
files are read like the reference entrypoint (main.go:20-60).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import sys
from typing import List, Optional

from .config.app_config import ApplicationConfig, parse_duration

ENV_FILES = [".env", "localai.env", os.path.expanduser("~/.config/localai.env"), "/etc/localai.env"]


def load_env_files():
    for p in ENV_FILES:
        try:
            with open(p) as f:
                for line in f:
                    line = line.strip()
                    if not line or line.startswith("#") or "=" not in line:
                        continue
                    k, v = line.split("=", 1)
                    k = k.strip().removeprefix("export ").strip()
                    v = v.strip().strip('"').strip("'")
                    os.environ.setdefault(k, v)
        except OSError:
            continue


# (flag, ApplicationConfig field, kind)
RUN_FLAGS = [
    ("--models-path", "models_path", str), ("--backend-assets-path", "backend_assets_path", str),
    ("--image-path", "image_dir", str), ("--audio-path", "audio_dir", str), ("--upload-path", "upload_dir", str),
    ("--config-path", "config_dir", str), ("--localai-config-dir", "dynamic_config_dir", str),
    ("--localai-config-dir-poll-interval", "dynamic_config_poll_interval", "duration"),
    ("--models-config-file", "models_config_file", str), ("--galleries", "galleries", "json"),
    ("--autoload-galleries", "autoload_galleries", bool), ("--remote-library", "remote_library", str),
    ("--preload-models", "preload_models", str), ("--models", "model_urls", "list"),
    ("--preload-models-config", "preload_models_from_path", str), ("--f16", "f16", bool),
    ("--threads", "threads", int), ("--context-size", "context_size", int), ("--address", "address", str),
    ("--cors", "cors", bool), ("--cors-allow-origins", "cors_allow_origins", str), ("--csrf", "csrf", bool),
    ("--upload-limit", "upload_limit_mb", int), ("--api-keys", "api_keys", "list"),
    ("--disable-webui", "disable_webui", bool), ("--disable-predownload-scan", "disable_predownload_scan", bool),
    ("--opaque-errors", "opaque_errors", bool), ("--use-subtle-key-comparison", "use_subtle_key_comparison", bool),
    ("--disable-api-key-requirement-for-http-get", "disable_api_key_requirement_for_http_get", bool),
    ("--http-get-exempted-endpoints", "http_get_exempted_endpoints", "list"), ("--p2p", "p2p", bool),
    ("--p2ptoken", "p2p_token", str), ("--p2p-network-id", "p2p_network_id", str),
    ("--parallel-requests", "parallel_backend_requests", bool),
    ("--single-active-backend", "single_active_backend", bool),
    ("--preload-backend-only", "preload_backend_only", bool),
    ("--external-grpc-backends", "external_grpc_backends", "backends"),
    ("--enable-watchdog-idle", "watchdog_idle", bool), ("--watchdog-idle-timeout", "watchdog_idle_timeout", "duration"),
    ("--enable-watchdog-busy", "watchdog_busy", bool), ("--watchdog-busy-timeout", "watchdog_busy_timeout", "duration"),
    ("--federated", "federated", bool), ("--disable-gallery-endpoint", "disable_gallery_endpoint", bool),
    ("--load-to-memory", "load_to_memory", "list"), ("--engine-mode", "engine_mode", str),
]


def _convert(kind, v):
    if kind is bool:
        return True if v is True else str(v).lower() in ("1", "true", "yes", "on")
    if kind is int:
        return int(v)
    if kind == "duration":
        return parse_duration(v)
    if kind == "json":
        return json.loads(v)
    if kind == "list":
        return [x for x in (v if isinstance(v, list) else str(v).split(",")) if x]
    if kind == "backends":
        out = {}
        for item in (v if isinstance(v, list) else str(v).split(",")):
            name, _, uri = item.partition(":")
            if name and uri:
                out[name] = uri
        return out
    return v


def add_run_flags(p: argparse.ArgumentParser):
    p.add_argument("models_args", nargs="*", help="model configuration URLs / gallery names to load")
    for flag, field, kind in RUN_FLAGS:
        if kind is bool:
            p.add_argument(flag, dest=field, nargs="?", const=True, default=None)
        else:
            p.add_argument(flag, dest=field, default=None)
    p.add_argument("--http-server", default="native", choices=["native", "uvicorn"])
    p.add_argument("--log-level", default=os.environ.get("LOCALAI_LOG_LEVEL", "info"))


def app_config_from_args(a) -> ApplicationConfig:
    cfg = ApplicationConfig.from_env()
    for flag, field, kind in RUN_FLAGS:
        v = getattr(a, field, None)
        if v is not None:
            setattr(cfg, field, _convert(kind, v))
    if getattr(a, "models_args", None):
        cfg.model_urls = list(cfg.model_urls) + list(a.models_args)
    return cfg


def parse_address(addr: str):
    host, _, port = addr.rpartition(":")
    return (host or "0.0.0.0"), int(port or 8080)


def cmd_run(a) -> int:
    from .startup import run_server, startup
    cfg = app_config_from_args(a)
    state = startup(cfg)
    if cfg.preload_backend_only:
        from .startup import load_to_memory
        asyncio.run(load_to_memory(state))
        return 0
    host, port = parse_address(cfg.address)
    run_server(state, host, port, a.http_server)
    return 0


def cmd_models(a) -> int:
    from . import gallery as gal
    cfg = ApplicationConfig.from_env()
    if a.models_path:
        cfg.models_path = a.models_path
    if a.galleries:
        cfg.galleries = json.loads(a.galleries)
    if a.action == "list":
        for m in gal.available_models(cfg.galleries, cfg.models_path):
            print(f"{'*' if m.installed else ' '} {m.id()}")
        return 0
    for name in a.names:
        gal.install_from_gallery(cfg.galleries, name, cfg.models_path, gal.GalleryModel())
        print(f"installed {name}")
    return 0


async def _one_shot(cfg: ApplicationConfig, model: str, backend: str, rpc: str, req):
    from .startup import startup
    state = startup(cfg)
    bc = state.config_for(model)
    if backend:
        bc.backend = backend
    lm = await state.manager.load(bc)
    try:
        return await getattr(lm.handle, rpc)(req)
    finally:
        await state.manager.stop_all()


def cmd_tts(a) -> int:
    from .grpc import backend_pb as pb
    cfg = ApplicationConfig.from_env(models_path=a.models_path or ApplicationConfig.from_env().models_path)
    out = os.path.abspath(a.output_file or "tts.wav")
    res = asyncio.run(_one_shot(cfg, a.model, a.backend, "TTS",
                                pb.TTSRequest(text=" ".join(a.text), model=a.model, dst=out, voice=a.voice or "",
                                              language=a.language or "")))
    print(out if res.success else res.message)
    return 0 if res.success else 1


def cmd_sound(a) -> int:
    from .grpc import backend_pb as pb
    cfg = ApplicationConfig.from_env(models_path=a.models_path or ApplicationConfig.from_env().models_path)
    out = os.path.abspath(a.output_file or "sound.wav")
    kw = {"text": " ".join(a.text), "model": a.model, "dst": out}
    if a.duration:
        kw["duration"] = float(a.duration)
    res = asyncio.run(_one_shot(cfg, a.model, a.backend, "SoundGeneration", pb.SoundGenerationRequest(**kw)))
    print(out if res.success else res.message)
    return 0 if res.success else 1


def cmd_transcript(a) -> int:
    from .grpc import backend_pb as pb
    cfg = ApplicationConfig.from_env(models_path=a.models_path or ApplicationConfig.from_env().models_path)
    res = asyncio.run(_one_shot(cfg, a.model, a.backend, "AudioTranscription",
                                pb.TranscriptRequest(dst=os.path.abspath(a.filename), language=a.language or "",
                                                     threads=int(a.threads or 4))))
    for s in res.segments:
        print(s.text)
    return 0


def _hf_scan(a, fetch=None) -> int:
    """core/cli/util.go:75-110 (best effort, HuggingFace only): scan the given URIs, or with none
    given every installed gallery model; exit 1 when a known-unsafe file is found."""
    from .utils.downloader import UnsafeFilesFound, hf_scan
    print("LocalAI Security Scanner - This is BEST EFFORT functionality! Currently limited to huggingface models!")
    bad = []
    if not a.file:
        from .gallery import safety_scan_gallery_models
        try:
            galleries = json.loads(a.galleries or "[]")
        except ValueError:
            print("unable to load galleries")
            galleries = []
        try:
            bad = safety_scan_gallery_models(galleries, a.models_path, fetch=fetch)
        except Exception as e:
            print(f"unable to list gallery models: {e}")
            return 1
    for uri in a.file:
        print(f"scanning specific uri {uri}")
        try:
            hf_scan(uri, fetch=fetch)
        except UnsafeFilesFound as e:
            bad.append({"uri": uri, "clamAV": e.result["clamAVInfectedFiles"], "pickles": e.result["dangerousPickles"]})
        except Exception as e:  # not an HF repo / scan unreachable: not a verdict (reference ignores it)
            print(f"scan skipped for {uri}: {e}")
    for b in bad:
        print(f"! WARNING ! A known-vulnerable model is included: {json.dumps(b)}")
    if not bad:
        print("No security warnings were detected for your installed models. Please note that this is a "
              "BEST EFFORT tool, and all issues may not be detected.")
    return 1 if bad else 0


def cmd_util(a) -> int:
    from .gguf import gguf_info
    if a.action == "hf-scan":
        return _hf_scan(a)
    if a.file and len(a.file) != 1:
        print(f"util {a.action}: exactly one file")
        return 2
    a.file = a.file[0] if a.file else ""
    if a.action == "gguf-info":
        info = gguf_info(a.file)
        print(json.dumps(info, indent=2, default=str))
        return 0
    if a.action == "usecase-heuristic":
        from .config.backend_config import USECASE_FLAGS
        from .config.loader import BackendConfigLoader
        ld = BackendConfigLoader(os.path.dirname(os.path.abspath(a.file)))
        ld.load_backend_config(a.file)
        for c in ld.all():
            flags = [n for n, f in USECASE_FLAGS.items() if f and c.guess_usecases(f)]
            print(f"{c.name}: {', '.join(flags) or 'none'}")
        return 0
    return 2


def cmd_federated(a) -> int:
    from .gateway.federated import FederatedBalancer, create_federated_app
    from .gateway.native_server import NativeHTTPServer
    workers = [w for w in (a.workers or os.environ.get("LOCALAI_FEDERATED_WORKERS", "")).split(",") if w]
    app = create_federated_app(FederatedBalancer(workers, "random" if a.random_worker else "least-used",
                                                 a.target_worker or ""))
    host, port = parse_address(a.address)
    NativeHTTPServer(app, host, port).run()
    return 0


def cmd_explorer(a) -> int:
    """`core/cli/explorer.go:22-49`: network directory + discovery (gateway/explorer.py)."""
    import threading

    from .gateway.explorer import Database, DiscoveryServer, create_explorer_app, parse_duration
    db = Database(a.pool_database)
    dur = parse_duration(a.connection_timeout)
    if a.only_sync:
        DiscoveryServer(db, dur, a.connection_error_threshold).start(keep_running=False)
        return 0
    if a.with_sync:
        ds = DiscoveryServer(db, dur, a.connection_error_threshold)
        threading.Thread(target=ds.start, name="explorer-sync", daemon=True).start()
    from .gateway.native_server import NativeHTTPServer
    host, port = parse_address(a.address)
    NativeHTTPServer(create_explorer_app(db), host, port).run()
    return 0


def cmd_worker(a) -> int:
    from .parallel.worker import main as worker_main
    rest = list(a.rest)
    if rest and rest[0] in ("tp", "llama-cpp-rpc", "p2p-llama-cpp-rpc"):  # reference command names
        rest = rest[1:]
    return worker_main(rest)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("local-ai", description="LocalAI-compatible server, MI355X-native engine")
    ap.add_argument("--log-level", default=None)
    sub = ap.add_subparsers(dest="cmd")
    add_run_flags(sub.add_parser("run", help="start the API server"))
    m = sub.add_parser("models", help="gallery models")
    m.add_argument("action", choices=["list", "install"])
    m.add_argument("names", nargs="*")
    m.add_argument("--models-path", default=None)
    m.add_argument("--galleries", default=None)
    for name, fn in (("tts", cmd_tts), ("sound-generation", cmd_sound)):
        t = sub.add_parser(name)
        t.add_argument("text", nargs="+")
        t.add_argument("--model", "-m", required=True)
        t.add_argument("--backend", "-b", default="")
        t.add_argument("--voice", default="")
        t.add_argument("--language", default="")
        t.add_argument("--duration", default=None)
        t.add_argument("--output-file", default=None)
        t.add_argument("--models-path", default=None)
        t.set_defaults(fn=fn)
    t = sub.add_parser("transcript")
    t.add_argument("filename")
    t.add_argument("--model", "-m", required=True)
    t.add_argument("--backend", "-b", default="")
    t.add_argument("--language", default="")
    t.add_argument("--threads", default=None)
    t.add_argument("--models-path", default=None)
    u = sub.add_parser("util")
    u.add_argument("action", choices=["gguf-info", "usecase-heuristic", "hf-scan"])
    u.add_argument("file", nargs="*", help="GGUF/config file, or the URIs to scan (hf-scan)")
    u.add_argument("--models-path", default=os.environ.get("LOCALAI_MODELS_PATH", os.environ.get("MODELS_PATH", "models")))
    u.add_argument("--galleries", default=os.environ.get("LOCALAI_GALLERIES", os.environ.get("GALLERIES", "[]")))
    f = sub.add_parser("federated", help="request-level load balancer over LocalAI instances")
    f.add_argument("--address", default=os.environ.get("LOCALAI_ADDRESS", ":8080"))
    f.add_argument("--workers", default="", help="comma-separated worker base URLs")
    f.add_argument("--random-worker", action="store_true")
    f.add_argument("--target-worker", default="")
    e = sub.add_parser("explorer", help="directory of LocalAI networks with worker discovery")
    env = os.environ.get
    e.add_argument("--address", default=env("LOCALAI_ADDRESS", env("ADDRESS", ":8080")))
    e.add_argument("--pool-database", default=env("LOCALAI_POOL_DATABASE", env("POOL_DATABASE", "explorer.json")))
    e.add_argument("--connection-timeout", default=env("LOCALAI_CONNECTION_TIMEOUT", env("CONNECTION_TIMEOUT", "2m")))
    e.add_argument("--connection-error-threshold", type=int,
                   default=int(env("LOCALAI_CONNECTION_ERROR_THRESHOLD", env("CONNECTION_ERROR_THRESHOLD", "3"))))
    e.add_argument("--with-sync", action="store_true",
                   default=env("LOCALAI_WITH_SYNC", env("WITH_SYNC", "")).lower() in ("1", "true"))
    e.add_argument("--only-sync", action="store_true",
                   default=env("LOCALAI_ONLY_SYNC", env("ONLY_SYNC", "")).lower() in ("1", "true"))
    w = sub.add_parser("worker", help="tensor-parallel engine worker group (replaces llama-cpp-rpc workers)")
    w.add_argument("rest", nargs=argparse.REMAINDER)
    return ap


def main(argv: Optional[List[str]] = None) -> int:
    load_env_files()
    ap = build_parser()
    a = ap.parse_args(argv)
    lvl = (getattr(a, "log_level", None) or os.environ.get("LOCALAI_LOG_LEVEL", "info")).upper()
    logging.basicConfig(level=getattr(logging, lvl, logging.INFO), format="%(asctime)s %(levelname)s %(name)s %(message)s")
    if a.cmd is None:
        ap.print_help()
        return 2
    fn = {"run": cmd_run, "models": cmd_models, "transcript": cmd_transcript, "util": cmd_util,
          "worker": cmd_worker, "federated": cmd_federated, "explorer": cmd_explorer}.get(a.cmd) or getattr(a, "fn", None)
    return fn(a)


if __name__ == "__main__":
    sys.exit(main())
