"""LocalAI-specific, Jina and ElevenLabs endpoints (`core/http/routes/{localai,jina,elevenlabs,health}.go`,
`core/http/endpoints/{localai,jina,elevenlabs}/*`)."""
from __future__ import annotations

import os
import time
import uuid

from fastapi import APIRouter, Request
from fastapi.responses import FileResponse, JSONResponse, Response

from .. import __version__
from ..config.backend_config import BackendConfig
from ..grpc import backend_pb as pb
from .metrics import CONTENT_TYPE
from .model_manager import (BARK_BACKENDS, ENGINE_BACKENDS, HF_BACKENDS, MAMBA_BACKEND, MUSICGEN_BACKENDS,
                            PARLER_BACKENDS, RWKV_BACKEND, SD_BACKENDS, STORE_BACKEND, VITS_BACKENDS)
from . import schema as sc
from .openai_routes import APIError, merge_request_with_config, model_from_context, read_request, typed_body


def build_router(state) -> APIRouter:
    r = APIRouter()

    async def ok():
        return Response(status_code=200)

    r.add_api_route("/healthz", ok, methods=["GET"])
    r.add_api_route("/readyz", ok, methods=["GET"])

    async def version():
        return {"version": __version__}

    r.add_api_route("/version", version, methods=["GET"])

    # ---------------------------------------------------------------- generated media
    # core/http/routes/openai.go:75,79: app.Static("/generated-images", ImageDir) and
    # ("/generated-audio", AudioDir) -- the URLs /v1/images/generations returns (response_format url)
    def _static(root_attr: str):
        async def serve(name: str):
            root = os.path.realpath(getattr(state.cfg, root_attr))
            p = os.path.realpath(os.path.join(root, name))
            if not p.startswith(root + os.sep) or not os.path.isfile(p):
                return JSONResponse({"error": {"code": 404, "message": "not found", "type": ""}}, status_code=404)
            return FileResponse(p)
        return serve

    r.add_api_route("/generated-images/{name:path}", _static("image_dir"), methods=["GET", "HEAD"])
    r.add_api_route("/generated-audio/{name:path}", _static("audio_dir"), methods=["GET", "HEAD"])

    async def system():
        backends = sorted(set(b for b in ENGINE_BACKENDS if b) | HF_BACKENDS | SD_BACKENDS | VITS_BACKENDS |
                          MUSICGEN_BACKENDS | BARK_BACKENDS | PARLER_BACKENDS | {MAMBA_BACKEND, RWKV_BACKEND}) + \
            [STORE_BACKEND] + list(state.cfg.external_grpc_backends)
        from ..utils.sysinfo import system_info
        return {"backends": backends, "loaded_models": [{"id": m.id} for m in state.manager.list_loaded()],
                "system": system_info()}

    r.add_api_route("/system", system, methods=["GET"])

    async def metrics():
        state.metrics.observe_engines(state.manager)
        return Response(state.metrics.render(), media_type=CONTENT_TYPE)

    if not state.cfg.disable_metrics:
        r.add_api_route("/metrics", metrics, methods=["GET"])

    # ---------------------------------------------------------------- tokenize / token metrics
    async def tokenize(request: Request):
        model, req = await read_request(request, state, schema=sc.TokenizeRequest)
        cfg = merge_request_with_config(state, model, req)
        lm = await state.manager.load(cfg)
        res = await lm.handle.TokenizeString(pb.PredictOptions(Prompt=str(req.get("content") or "")))
        return {"tokens": list(res.tokens)}

    r.add_api_route("/v1/tokenize", tokenize, methods=["POST"], openapi_extra=sc.body_doc(sc.TokenizeRequest))

    async def token_metrics(request: Request):
        model, req = await read_request(request, state, schema=sc.TokenMetricsRequest)
        cfg = merge_request_with_config(state, model, req)
        lm = await state.manager.load(cfg)
        res = await lm.handle.GetMetrics(pb.MetricsRequest())
        return {"slot_id": res.slot_id, "prompt_json_for_slot": res.prompt_json_for_slot,
                "tokens_per_second": res.tokens_per_second, "tokens_generated": res.tokens_generated,
                "prompt_tokens_processed": res.prompt_tokens_processed}

    r.add_api_route("/v1/tokenMetrics", token_metrics, methods=["GET", "POST"])

    # ---------------------------------------------------------------- backend monitor
    def _find_loaded(name: str):
        lm = state.manager.get(name)
        if lm is None:
            cfg = state.configs.get(name)
            if cfg is not None:
                lm = state.manager.get(cfg.name)
        return lm

    async def monitor(request: Request):
        try:
            body = await request.json()
        except Exception:
            body = {}
        name = (body or {}).get("model") or request.query_params.get("model", "")
        lm = _find_loaded(name)
        if lm is None:
            raise APIError(f"backend {name} is not currently loaded", 500)
        try:
            st = await lm.handle.Status(pb.HealthMessage())
            out = {"state": int(st.state), "memory": {"total": st.memory.total,
                                                       "breakdown": dict(st.memory.breakdown)}}
            if hasattr(lm.handle, "stats"):  # data-parallel replicas: per-replica load
                out["replicas"] = lm.handle.stats()
            return out
        except Exception:
            import psutil
            p = psutil.Process(lm.process.pid) if getattr(lm.process, "pid", None) else psutil.Process()
            mi = p.memory_info()
            return {"MemoryInfo": {"rss": mi.rss, "vms": mi.vms}, "MemoryPercent": p.memory_percent(),
                    "CPUPercent": p.cpu_percent(interval=None)}

    async def backend_shutdown(request: Request):
        try:
            body = await request.json()
        except Exception:
            body = {}
        name = (body or {}).get("model", "")
        lm = _find_loaded(name)
        if lm is None:
            raise APIError(f"backend {name} is not currently loaded", 500)
        await state.manager.shutdown(lm.id)
        return Response(status_code=200)

    r.add_api_route("/backend/monitor", monitor, methods=["GET"])
    r.add_api_route("/backend/shutdown", backend_shutdown, methods=["POST"])

    # ---------------------------------------------------------------- stores
    async def _store(name: str):
        cfg = BackendConfig({"name": name or "default", "backend": STORE_BACKEND,
                             "parameters": {"model": name or "default"}})
        return await state.manager.load(cfg)

    def _keys(ks):
        return [pb.StoresKey(Floats=[float(x) for x in k]) for k in (ks or [])]

    async def stores_set(request: Request):
        b = await typed_body(request, sc.StoresSet)
        keys, vals = b.get("keys") or [], b.get("values") or []
        if len(keys) != len(vals):
            raise APIError("keys and values must have the same length", 400)
        lm = await _store(b.get("store", ""))
        res = await lm.handle.StoresSet(pb.StoresSetOptions(
            Keys=_keys(keys), Values=[pb.StoresValue(Bytes=str(v).encode()) for v in vals]))
        if not res.success:
            raise APIError(res.message, 500)
        return Response(status_code=200)

    async def stores_delete(request: Request):
        b = await typed_body(request, sc.StoresDelete)
        lm = await _store(b.get("store", ""))
        res = await lm.handle.StoresDelete(pb.StoresDeleteOptions(Keys=_keys(b.get("keys"))))
        if not res.success:
            raise APIError(res.message, 500)
        return Response(status_code=200)

    async def stores_get(request: Request):
        b = await typed_body(request, sc.StoresGet)
        lm = await _store(b.get("store", ""))
        res = await lm.handle.StoresGet(pb.StoresGetOptions(Keys=_keys(b.get("keys"))))
        return {"keys": [list(k.Floats) for k in res.Keys],
                "values": [bytes(v.Bytes).decode("utf-8", "replace") for v in res.Values]}

    async def stores_find(request: Request):
        b = await typed_body(request, sc.StoresFind)
        lm = await _store(b.get("store", ""))
        res = await lm.handle.StoresFind(pb.StoresFindOptions(Key=pb.StoresKey(Floats=b.get("key") or []),
                                                              TopK=int(b.get("topk") or 0)))
        return {"keys": [list(k.Floats) for k in res.Keys],
                "values": [bytes(v.Bytes).decode("utf-8", "replace") for v in res.Values],
                "similarities": list(res.Similarities)}

    for path, fn, m in (("set", stores_set, sc.StoresSet), ("delete", stores_delete, sc.StoresDelete),
                        ("get", stores_get, sc.StoresGet), ("find", stores_find, sc.StoresFind)):
        r.add_api_route(f"/stores/{path}", fn, methods=["POST"], openapi_extra=sc.body_doc(m))

    # ---------------------------------------------------------------- rerank (Jina)
    async def rerank(request: Request):
        model, req = await read_request(request, state, schema=sc.JINARerankRequest)
        cfg = merge_request_with_config(state, model, req)
        lm = await state.manager.load(cfg)
        res = await lm.handle.Rerank(pb.RerankRequest(query=str(req.get("query") or ""),
                                                      documents=[str(d) for d in req.get("documents") or []],
                                                      top_n=int(req.get("top_n") or 0)))
        return {"model": req.get("model", model),
                "usage": {"total_tokens": res.usage.total_tokens, "prompt_tokens": res.usage.prompt_tokens},
                "results": [{"index": d.index, "document": {"text": d.text}, "relevance_score": d.relevance_score}
                            for d in res.results]}

    r.add_api_route("/v1/rerank", rerank, methods=["POST"], openapi_extra=sc.body_doc(sc.JINARerankRequest))

    # ---------------------------------------------------------------- TTS / sound generation
    async def _tts(model: str, backend: str, text: str, voice: str, language: str):
        cfg = merge_request_with_config(state, model, {"model": model})
        if backend:
            cfg.backend = backend
        elif not cfg.backend:
            cfg.backend = "piper"  # core/backend/tts.go: piper when neither the request nor the config names one
        lm = await state.manager.load(cfg)
        os.makedirs(state.cfg.audio_dir, exist_ok=True)
        dst = os.path.join(state.cfg.audio_dir, f"tts_{uuid.uuid4().hex}.wav")
        res = await lm.handle.TTS(pb.TTSRequest(text=text, model=cfg.model_file_name(), dst=dst, voice=voice,
                                                language=language))
        if not res.success:
            raise APIError(res.message, 500)
        return FileResponse(dst, media_type="audio/wav")

    async def tts(request: Request):
        b = await typed_body(request, sc.TTSRequest)
        model = model_from_context(request, state, b.get("model", ""), False)
        return await _tts(model, b.get("backend", ""), b.get("input", ""), b.get("voice", ""), b.get("language", ""))

    async def tts_eleven(request: Request, voice_id: str):
        b = await typed_body(request, sc.ElevenLabsTTSRequest)
        model = model_from_context(request, state, b.get("model_id", ""), False)
        return await _tts(model, "", b.get("text", ""), voice_id, "")

    async def sound_generation(request: Request):
        b = await typed_body(request, sc.ElevenLabsSoundGenerationRequest)
        model = model_from_context(request, state, b.get("model_id", ""), False)
        cfg = merge_request_with_config(state, model, {"model": model})
        lm = await state.manager.load(cfg)
        os.makedirs(state.cfg.audio_dir, exist_ok=True)
        dst = os.path.join(state.cfg.audio_dir, f"sound_{uuid.uuid4().hex}.wav")
        kw = {"text": b.get("text", ""), "model": cfg.model_file_name(), "dst": dst}
        if b.get("duration_seconds") is not None:
            kw["duration"] = float(b["duration_seconds"])
        if b.get("prompt_influence") is not None:
            kw["temperature"] = float(b["prompt_influence"])
        if b.get("do_sample") is not None:
            kw["sample"] = bool(b["do_sample"])
        res = await lm.handle.SoundGeneration(pb.SoundGenerationRequest(**kw))
        if not res.success:
            raise APIError(res.message, 500)
        return FileResponse(dst, media_type="audio/wav")

    r.add_api_route("/tts", tts, methods=["POST"], openapi_extra=sc.body_doc(sc.TTSRequest))
    r.add_api_route("/v1/audio/speech", tts, methods=["POST"], openapi_extra=sc.body_doc(sc.TTSRequest))
    r.add_api_route("/v1/text-to-speech/{voice_id}", tts_eleven, methods=["POST"],
                    openapi_extra=sc.body_doc(sc.ElevenLabsTTSRequest))
    r.add_api_route("/v1/sound-generation", sound_generation, methods=["POST"],
                    openapi_extra=sc.body_doc(sc.ElevenLabsSoundGenerationRequest))

    return r
