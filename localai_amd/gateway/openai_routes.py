"""OpenAI-compatible endpoints (`core/http/endpoints/openai/*`, routes `core/http/routes/openai.go`).

Per-request ids/timestamps (the reference shares them across requests: SURVEY Q1/Q2); SSE
framing `data: {json}\\n\\n` ... `data: [DONE]` as in chat.go:463-508; token-granular streaming
(the reference streams per UTF-8 rune, Q3); real usage counts in every stream chunk.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
import uuid
from typing import List

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, StreamingResponse

from .. import functions as fn
from ..config.backend_config import FLAG_CHAT, FLAG_COMPLETION, FLAG_EMBEDDINGS
from ..config.loader import build_name_filter, build_usecase_filter
from ..templates import CHAT_MESSAGE, CHAT_PROMPT, COMPLETION_PROMPT, EDIT_PROMPT
from . import schema as sc
from .inference import Inference, TokenUsage, finetune, update_request_config

log = logging.getLogger("localai_amd.api")
_DOC = sc.body_doc(sc.OpenAIRequest)


def _sse(obj) -> bytes:
    return b"data: " + json.dumps(obj, ensure_ascii=False, separators=(",", ":")).encode() + b"\n\n"


def _usage(u: TokenUsage) -> dict:
    return {"prompt_tokens": u.prompt, "completion_tokens": u.completion, "total_tokens": u.prompt + u.completion}


class APIError(Exception):
    def __init__(self, msg: str, code: int = 500):
        super().__init__(msg)
        self.code = code


async def typed_body(request: Request, model=sc.OpenAIRequest) -> dict:
    """The JSON body, checked against its request struct (gateway/schema.py): a field of the
    wrong type is a 400, as the reference's struct decoding makes it."""
    try:
        body = await request.json()
    except Exception:
        body = {}
    try:
        return sc.validate(model, body)
    except sc.SchemaError as e:
        raise APIError(str(e), 400)


async def read_request(request: Request, state, first_model: bool = True, path_model: str = "",
                       schema=sc.OpenAIRequest):
    body = await typed_body(request, schema)
    body["_correlation_id"] = request.headers.get("X-Correlation-ID") or str(uuid.uuid4())
    model = model_from_context(request, state, body.get("model", ""), first_model, path_model)
    return model, body


def model_from_context(request: Request, state, model_input: str, first_model: bool, path_model: str = "") -> str:
    """core/http/ctx/fiber.go:18-47 (path param > query > body; bearer naming a model file wins)."""
    if path_model:
        model_input = path_model
    q = request.query_params.get("model")
    if q:
        model_input = q
    auth = request.headers.get("authorization", "")
    bearer = auth.lstrip("Bear ") if auth else ""  # (sic) TrimLeft cutset semantics
    bearer_exists = bool(bearer) and state.exists_in_model_path(bearer)
    if not model_input and not bearer_exists and first_model:
        models = state.list_models()
        if not models:
            raise APIError("no model specified", 400)
        model_input = models[0]
    if bearer_exists:
        model_input = bearer
    return model_input


def merge_request_with_config(state, model_name: str, body: dict):
    cfg = state.config_for(model_name)
    update_request_config(cfg, body)
    if not cfg.validate():
        raise APIError("failed to validate config", 400)
    return cfg


def build_router(state) -> APIRouter:
    r = APIRouter()

    # ------------------------------------------------------------------------ chat
    async def chat(request: Request):
        cid = str(uuid.uuid4())
        created = int(time.time())
        model, req = await read_request(request, state)
        cfg = merge_request_with_config(state, model, req)
        funcs = list(req.get("_functions") or [])
        should_use_fn = len(funcs) > 0 and cfg.should_use_functions()
        strict = any(f.get("strict") for f in funcs)
        fcfg = cfg.functions
        no_action = fcfg.get("no_action_function_name") or "answer"
        no_action_desc = fcfg.get("no_action_description_name") or \
            "use this action to answer without performing any action"
        gopts = fn.grammar_options(fcfg)
        grammar = req.get("grammar") or ""
        rf = cfg.response_format_map
        if rf:
            if rf.get("type") == "json_object":
                grammar = fn.JSON_BNF
            elif rf.get("type") == "json_schema":
                schema = ((rf.get("json_schema") or {}).get("schema")) or {}
                try:
                    grammar = fn.structure_grammar({"anyOf": [schema]}, gopts)
                except Exception as e:
                    log.debug("json_schema grammar failed: %s", e)
        cfg.raw["grammar"] = grammar
        disable_grammar = bool((fcfg.get("grammar") or {}).get("disable"))
        if (not disable_grammar or strict) and should_use_fn:
            if not fcfg.get("disable_no_action"):
                funcs.append({"name": no_action, "description": no_action_desc, "parameters": {
                    "properties": {"message": {"type": "string", "description": "The message to reply the user with"}}}})
            if cfg.function_to_call():
                funcs = fn.select(funcs, cfg.function_to_call())
            nk = fcfg.get("function_name_key") or ""
            js = fn.to_json_structure(funcs, nk, nk)
            try:
                cfg.raw["grammar"] = fn.structure_grammar(js, gopts)
            except Exception as e:
                log.debug("function grammar failed: %s", e)
        elif req.get("grammar_json_functions"):
            try:
                cfg.raw["grammar"] = fn.structure_grammar(req["grammar_json_functions"], gopts)
            except Exception:
                pass
        elif cfg.function_to_call():
            funcs = fn.select(funcs, cfg.function_to_call())

        pred_input = ""
        tpl = cfg.template
        if not tpl.get("use_tokenizer_template") or should_use_fn:
            suppress_sys = False
            mess: List[str] = []
            msgs = req.get("messages") or []
            for idx, m in enumerate(msgs):
                role = m.get("role", "")
                if (m.get("function_call") is not None or m.get("tool_calls") is not None) and role == "assistant":
                    if cfg.roles.get("assistant_function_call"):
                        role = "assistant_function_call"
                rname = cfg.roles.get(role, "")
                sc = m.get("_string_content", "")
                content_exists = m.get("content") is not None and sc != ""
                fcall = m.get("function_call")
                if m.get("tool_calls"):
                    fcall = m["tool_calls"]
                content = ""
                if tpl.get("chat_message"):
                    data = {"SystemPrompt": cfg.system_prompt, "Role": rname, "RoleName": role, "Content": sc,
                            "FunctionCall": fcall, "FunctionName": m.get("name", "") or "",
                            "LastMessage": idx == len(msgs) - 1,
                            "Function": bool(cfg.raw.get("grammar")) and idx == len(msgs) - 1, "MessageIndex": idx}
                    try:
                        out = state.templates.evaluate(CHAT_MESSAGE, tpl["chat_message"], data)
                        if out == "":
                            continue
                        content = out
                    except Exception as e:
                        log.error("error processing message with template, skipping: %s", e)
                if content == "":
                    def marshal(v, with_role):
                        j = fn._go_json(v)
                        nonlocal content
                        piece = f"{rname} {j}" if with_role else j
                        content = (content + "\n" + piece) if content_exists else piece
                    if rname:
                        if content_exists:
                            content = f"{rname}{sc}"
                        if m.get("function_call") is not None:
                            marshal(m["function_call"], True)
                        if m.get("tool_calls") is not None:
                            marshal(m["tool_calls"], True)
                    else:
                        if content_exists:
                            content = sc
                        if m.get("function_call") is not None:
                            marshal(m["function_call"], False)
                        if m.get("tool_calls") is not None:
                            marshal(m["tool_calls"], False)
                    if content_exists and role == "system":
                        suppress_sys = True
                mess.append(content)
            join = tpl.get("join_chat_messages_by_character")
            pred_input = ("\n" if join is None else join).join(mess)
            template_file = ""
            if state.exists_in_model_path(f"{cfg.model}.tmpl"):
                template_file = cfg.model
            if tpl.get("chat") and not should_use_fn:
                template_file = tpl["chat"]
            if tpl.get("function") and should_use_fn:
                template_file = tpl["function"]
            if template_file:
                try:
                    pred_input = state.templates.evaluate(CHAT_PROMPT, template_file, {
                        "SystemPrompt": cfg.system_prompt, "SuppressSystemPrompt": suppress_sys,
                        "Input": pred_input, "Functions": funcs, "Instruction": "", "MessageIndex": 0})
                except Exception as e:
                    log.debug("template failed loading: %s", e)
        inf = Inference(state, cfg, req, "chat")
        model_out = req.get("model", model)
        headers = {"X-Correlation-ID": req["_correlation_id"]}

        if req.get("stream") and not should_use_fn:
            h = await _native_stream(request, state, cfg, req, pred_input, cid, created, model_out, "chat")
            if h is not None:
                return h

        if req.get("stream"):
            async def gen_plain():
                first = {"id": cid, "created": created, "model": model_out, "object": "chat.completion.chunk",
                         "choices": [{"index": 0, "finish_reason": None,
                                      "delta": {"role": "assistant", "content": ""}}]}
                yield _sse(first)
                usage = TokenUsage()
                try:
                    async for text, usage, final in inf.stream(pred_input):
                        if final:
                            break
                        yield _sse({"id": cid, "created": created, "model": model_out,
                                    "object": "chat.completion.chunk",
                                    "choices": [{"index": 0, "finish_reason": None, "delta": {"content": text}}],
                                    "usage": _usage(usage)})
                except Exception as e:
                    yield _sse({"error": {"message": str(e), "type": "server_error", "code": 500}})
                yield _sse({"id": cid, "created": created, "model": model_out, "object": "chat.completion.chunk",
                            "choices": [{"index": 0, "finish_reason": "stop", "delta": {"content": ""}}],
                            "usage": _usage(usage)})
                yield b"data: [DONE]\n\n"

            async def gen_tools():
                result = ""
                usage = TokenUsage()
                async for text, usage, final in inf.stream(pred_input):
                    result += text
                text_content = fn.parse_text_content(result, fcfg)
                res = fn.cleanup_llm_result(result, fcfg)
                calls = fn.parse_function_call(res, fcfg)
                tools_called = False
                if not calls or calls[0].name == no_action:
                    yield _sse({"id": cid, "created": created, "model": model_out, "object": "chat.completion.chunk",
                                "choices": [{"index": 0, "finish_reason": None,
                                             "delta": {"role": "assistant", "content": text_content}}]})
                    answer = await handle_question(state, cfg, req, calls, res, pred_input)
                    yield _sse({"id": cid, "created": created, "model": model_out, "object": "chat.completion.chunk",
                                "choices": [{"index": 0, "finish_reason": None, "delta": {"content": answer}}],
                                "usage": _usage(usage)})
                else:
                    tools_called = True
                    for i, c in enumerate(calls):
                        yield _sse({"id": cid, "created": created, "model": model_out,
                                    "object": "chat.completion.chunk", "choices": [{"index": 0, "finish_reason": None,
                                    "delta": {"role": "assistant", "tool_calls": [{
                                        "index": i, "id": cid, "type": "function",
                                        "function": {"name": c.name, "arguments": ""}}]}}]})
                        yield _sse({"id": cid, "created": created, "model": model_out,
                                    "object": "chat.completion.chunk", "choices": [{"index": 0, "finish_reason": None,
                                    "delta": {"role": "assistant", "content": text_content, "tool_calls": [{
                                        "index": i, "id": cid, "type": "function",
                                        "function": {"arguments": c.arguments}}]}}]})
                finish = "tool_calls" if tools_called else "stop"
                yield _sse({"id": cid, "created": created, "model": model_out, "object": "chat.completion.chunk",
                            "choices": [{"index": 0, "finish_reason": finish, "delta": {"content": text_content}}],
                            "usage": _usage(usage)})
                yield b"data: [DONE]\n\n"

            return StreamingResponse(gen_tools() if should_use_fn else gen_plain(), media_type="text/event-stream",
                                     headers={**headers, "Cache-Control": "no-cache", "Connection": "keep-alive"})

        n = max(1, int(req.get("n") or 1))
        choices = []
        usage = TokenUsage()
        for _ in range(n):
            text, u = await inf.predict(pred_input)
            usage.prompt += u.prompt
            usage.completion += u.completion
            s = finetune(cfg, pred_input, text)
            if not should_use_fn:
                choices.append({"index": 0, "finish_reason": "stop", "message": {"role": "assistant", "content": s}})
                continue
            text_content = fn.parse_text_content(s, fcfg)
            s2 = fn.cleanup_llm_result(s, fcfg)
            calls = fn.parse_function_call(s2, fcfg)
            if not calls or calls[0].name == no_action:
                answer = await handle_question(state, cfg, req, calls, s2, pred_input)
                choices.append({"index": 0, "finish_reason": "stop",
                                "message": {"role": "assistant", "content": answer}})
            else:
                tool_choice = {"index": 0, "finish_reason": "tool_calls" if req.get("tools") else "",
                               "message": {"role": "assistant"}}
                for c in calls:
                    if req.get("tools"):
                        tool_choice["message"]["content"] = text_content
                        tool_choice["message"].setdefault("tool_calls", []).append(
                            {"index": 0, "id": cid, "type": "function",
                             "function": {"name": c.name, "arguments": c.arguments}})
                    else:
                        choices.append({"index": 0, "finish_reason": "function_call", "message": {
                            "role": "assistant", "content": text_content,
                            "function_call": {"name": c.name, "arguments": c.arguments}}})
                if req.get("tools"):
                    choices.append(tool_choice)
        return JSONResponse({"id": cid, "created": created, "model": model_out, "object": "chat.completion",
                             "choices": choices, "usage": _usage(usage)}, headers=headers)

    for p in ("/v1/chat/completions", "/chat/completions"):
        r.add_api_route(p, chat, methods=["POST"], openapi_extra=_DOC)
    # endpoints that read only the Request: the native server may call them without Starlette's
    # router (app.create_app composes the same middleware and error handlers around them)
    r.native_fast = {p: chat for p in ("/v1/chat/completions", "/chat/completions")}

    # ------------------------------------------------------------------------ completion
    async def completion(request: Request, model_path: str = ""):
        cid = str(uuid.uuid4())
        created = int(time.time())
        model, req = await read_request(request, state, path_model=model_path)
        cfg = merge_request_with_config(state, model, req)
        rf = cfg.response_format_map
        grammar = req.get("grammar") or ""
        if rf and rf.get("type") == "json_object":
            grammar = fn.JSON_BNF
        cfg.raw["grammar"] = grammar
        template_file = ""
        if state.exists_in_model_path(f"{cfg.model}.tmpl"):
            template_file = cfg.model
        if cfg.template.get("completion"):
            template_file = cfg.template["completion"]
        model_out = req.get("model", model)
        inf = Inference(state, cfg, req, "completion")

        def apply_tpl(s):
            if not template_file:
                return s
            try:
                return state.templates.evaluate(COMPLETION_PROMPT, template_file,
                                                {"Input": s, "SystemPrompt": cfg.system_prompt})
            except Exception:
                return s

        if req.get("stream"):
            if len(cfg.prompt_strings) > 1:
                raise APIError("cannot handle more than 1 `PromptStrings` when Streaming", 400)
            pred_input = apply_tpl(cfg.prompt_strings[0] if cfg.prompt_strings else "")
            h = await _native_stream(request, state, cfg, req, pred_input, cid, created, model_out, "completion")
            if h is not None:
                return h

            async def gen():
                usage = TokenUsage()
                async for text, usage, final in inf.stream(pred_input):
                    if final:
                        break
                    yield _sse({"id": cid, "created": created, "model": model_out, "object": "text_completion",
                                "choices": [{"index": 0, "text": text, "finish_reason": None}],
                                "usage": _usage(usage)})
                yield _sse({"id": cid, "created": created, "model": model_out, "object": "text_completion",
                            "choices": [{"index": 0, "finish_reason": "stop", "text": ""}], "usage": _usage(usage)})
                yield b"data: [DONE]\n\n"
            return StreamingResponse(gen(), media_type="text/event-stream",
                                     headers={"X-Correlation-ID": cid, "Cache-Control": "no-cache"})
        choices = []
        usage = TokenUsage()
        for k, p in enumerate(cfg.prompt_strings or [""]):
            pi = apply_tpl(p)
            for _ in range(max(1, int(req.get("n") or 1))):
                text, u = await inf.predict(pi)
                usage.prompt += u.prompt
                usage.completion += u.completion
                choices.append({"index": k, "finish_reason": "stop", "text": finetune(cfg, pi, text)})
        return JSONResponse({"id": cid, "created": created, "model": model_out, "object": "text_completion",
                             "choices": choices, "usage": _usage(usage)}, headers={"X-Correlation-ID": cid})

    async def completion_engine(request: Request, model: str):
        return await completion(request, model_path=model)

    for p in ("/v1/completions", "/completions"):
        r.add_api_route(p, completion, methods=["POST"], openapi_extra=_DOC)
    r.native_fast.update({p: completion for p in ("/v1/completions", "/completions")})
    r.add_api_route("/v1/engines/{model}/completions", completion_engine, methods=["POST"])

    # ------------------------------------------------------------------------ edits
    async def edit(request: Request):
        cid = str(uuid.uuid4())
        created = int(time.time())
        model, req = await read_request(request, state)
        cfg = merge_request_with_config(state, model, req)
        template_file = ""
        if state.exists_in_model_path(f"{cfg.model}.tmpl"):
            template_file = cfg.model
        if cfg.template.get("edit"):
            template_file = cfg.template["edit"]
        inf = Inference(state, cfg, req, "edit")
        choices, usage = [], TokenUsage()
        for i in cfg.input_strings:
            pi = i
            if template_file:
                try:
                    pi = state.templates.evaluate(EDIT_PROMPT, template_file, {
                        "Input": i, "Instruction": req.get("instruction", ""), "SystemPrompt": cfg.system_prompt})
                except Exception:
                    pass
            text, u = await inf.predict(pi)
            usage.prompt += u.prompt
            usage.completion += u.completion
            choices.append({"index": 0, "text": finetune(cfg, pi, text)})
        return JSONResponse({"id": cid, "created": created, "model": req.get("model", model), "object": "edit",
                             "choices": choices, "usage": _usage(usage)})

    for p in ("/v1/edits", "/edits"):
        r.add_api_route(p, edit, methods=["POST"], openapi_extra=_DOC)

    # ------------------------------------------------------------------------ embeddings
    async def embeddings(request: Request, model_path: str = ""):
        from ..grpc import backend_pb as pb
        cid = str(uuid.uuid4())
        created = int(time.time())
        model, req = await read_request(request, state, path_model=model_path)
        cfg = merge_request_with_config(state, model, req)
        lm = await state.manager.load(cfg)
        items = []
        k = 0
        ptoks = 0
        for toks in cfg.input_tokens:
            res = await lm.handle.Embedding(pb.PredictOptions(EmbeddingTokens=toks))
            items.append({"embedding": _strip_trailing_zeros(list(res.embeddings)), "index": k, "object": "embedding"})
            k += 1
            ptoks += len(toks)
        for s in cfg.input_strings:
            res = await lm.handle.Embedding(pb.PredictOptions(Embeddings=s))
            items.append({"embedding": _strip_trailing_zeros(list(res.embeddings)), "index": k, "object": "embedding"})
            k += 1
        return JSONResponse({"object": "list", "created": created, "id": cid, "model": req.get("model", model),
                             "data": items, "usage": {"prompt_tokens": ptoks, "completion_tokens": 0,
                                                      "total_tokens": ptoks}})

    async def embeddings_engine(request: Request, model: str):
        return await embeddings(request, model_path=model)

    for p in ("/v1/embeddings", "/embeddings"):
        r.add_api_route(p, embeddings, methods=["POST"], openapi_extra=_DOC)
    r.add_api_route("/v1/engines/{model}/embeddings", embeddings_engine, methods=["POST"])

    # ------------------------------------------------------------------------ models
    async def list_models(request: Request):
        flt = build_name_filter(request.query_params.get("filter", ""))
        exclude = request.query_params.get("excludeConfigured", "").lower() in ("1", "true")
        from .state import ALWAYS_INCLUDE, SKIP_IF_CONFIGURED
        names = state.list_models(flt, SKIP_IF_CONFIGURED if exclude else ALWAYS_INCLUDE)
        seen, data = set(), []
        for n in names:
            if n in seen:
                continue
            seen.add(n)
            data.append({"id": n, "object": "model"})
        return {"object": "list", "data": data}

    for p in ("/v1/models", "/models"):
        r.add_api_route(p, list_models, methods=["GET"])

    # ------------------------------------------------------------------------ audio / images (external backends)
    async def transcription(request: Request):
        from ..grpc import backend_pb as pb
        import os
        import tempfile
        from ..utils.multipart import read_form
        form = await read_form(request)
        model = model_from_context(request, state, form.get("model", ""), True)
        cfg = merge_request_with_config(state, model, {})
        up = form.get("file")
        if up is None:
            raise APIError("file is required", 400)
        tmpdir = tempfile.mkdtemp()
        dst = os.path.join(tmpdir, os.path.basename(up.filename or "audio"))
        with open(dst, "wb") as f:
            f.write(await up.read())
        lm = await state.manager.load(cfg)
        res = await lm.handle.AudioTranscription(pb.TranscriptRequest(dst=dst, language=form.get("language", ""),
                                                                      threads=int(cfg.raw.get("threads") or 4)))
        return {"segments": [{"id": s.id, "start": s.start, "end": s.end, "text": s.text, "tokens": list(s.tokens)}
                             for s in res.segments], "text": res.text}

    r.add_api_route("/v1/audio/transcriptions", transcription, methods=["POST"])

    async def images(request: Request):
        from ..grpc import backend_pb as pb
        import base64
        import os
        import uuid as _u
        model, req = await read_request(request, state, first_model=False)
        if not model:
            model = "stablediffusion"
        cfg = merge_request_with_config(state, model, req)
        size = req.get("size") or "512x512"
        w, _, h = size.partition("x")
        prompt = str(req.get("prompt") or "")
        pos, _, neg = prompt.partition("|")
        os.makedirs(state.cfg.image_dir, exist_ok=True)
        out = []
        lm = await state.manager.load(cfg)
        for _ in range(max(1, int(req.get("n") or 1))):
            name = f"b64{_u.uuid4().hex}.png"
            dst = os.path.join(state.cfg.image_dir, name)
            res = await lm.handle.GenerateImage(pb.GenerateImageRequest(
                width=int(w or 512), height=int(h or 512), mode=int(req.get("mode") or 0), step=int(req.get("step") or 15),
                seed=int(req.get("seed") or 0), positive_prompt=pos, negative_prompt=neg, dst=dst,
                src=str(req.get("file") or "")))
            if res is not None and not getattr(res, "success", True):
                raise APIError(res.message or "image generation failed", 500)
            if req.get("response_format") == "b64_json":
                with open(dst, "rb") as f:
                    out.append({"b64_json": base64.b64encode(f.read()).decode()})
            else:
                base = str(request.base_url).rstrip("/")
                out.append({"url": f"{base}/generated-images/{name}"})
        return {"created": int(time.time()), "id": str(uuid.uuid4()), "data": out}

    r.add_api_route("/v1/images/generations", images, methods=["POST"], openapi_extra=_DOC)
    return r


async def _native_stream(request, state, cfg, req, pred_input: str, cid: str, created: int, model_out: str,
                         kind: str):
    """Token streaming without the event loop: bind a native SseSink (native/http_server.cpp) to
    the connection and hand it to the in-process engine.  Only the final event comes back to
    Python (once per request).  Returns None when not applicable (uvicorn, out-of-process or
    external backend), so the generic async-generator path is used instead."""
    nc = request.scope.get("localai.native")
    if nc is None:
        return None
    lm = await state.manager.load(cfg)
    sv = lm.servicer
    eng = getattr(sv, "engine", None) if sv is not None else None
    if eng is None or (getattr(eng, "clip", None) is not None and any(m.get("_images") for m in req.get("messages") or [])):
        return None  # images go through the generic path (the servicer hands them to the engine)
    from ..native import http
    from .inference import predict_options
    from .native_server import NativeHandledResponse
    po = predict_options(cfg, pred_input, req.get("messages"), state.models_path)
    po.CorrelationId = req.get("_correlation_id", "")
    pick = getattr(lm.handle, "pick_native", None)
    rep = None
    if pick is not None:
        # data-parallel replicas: the balancer picks; a remote pick takes the generic RPC path
        rep, sv = pick(po)
        if sv is None:
            return None
        eng = sv.engine
    prompt = sv._prompt(po)
    params = sv._params(po)
    obj = "chat.completion.chunk" if kind == "chat" else "text_completion"
    base = 'data: {"id":%s,"created":%d,"model":%s,"object":"%s","choices":[{"index":0,"finish_reason":' % (
        json.dumps(cid), created, json.dumps(model_out, ensure_ascii=False), obj)
    if kind == "chat":
        head, mid = base + 'null,"delta":{"content":"', '"}}],"usage":'
        fin_body = ',"delta":{"content":""}}],"usage":'
    else:
        head, mid = base + 'null,"text":"', '"}],"usage":'
        fin_body = ',"text":""}],"usage":'
    srv, conn = nc.srv, nc.conn
    srv.stream_start(conn, 200, [("content-type", "text/event-stream"), ("cache-control", "no-cache"),
                                 ("connection", "keep-alive"), ("x-correlation-id", req["_correlation_id"])])
    if kind == "chat":
        srv.stream_write(conn, (base + 'null,"delta":{"role":"assistant","content":""}}]}\n\n').encode())
    sink = http().SseSink(srv, conn, head.encode(), mid.encode(), b"}\n\n", 0)
    nc.handled = True
    loop = asyncio.get_running_loop()
    mid_ = lm.id
    metrics = state.metrics
    state.manager.mark_busy(mid_, True)
    t0 = time.perf_counter()

    def on_final(ev):  # engine thread, once per request
        if ev.text:
            sink.push(ev.text, ev.completion_tokens)
        if ev.error:
            err = json.dumps({"error": {"message": ev.error, "type": "server_error", "code": 500}})
            sink.finish(f"data: {err}\n\ndata: [DONE]\n\n".encode())
        else:
            usage = json.dumps({"prompt_tokens": ev.prompt_tokens, "completion_tokens": ev.completion_tokens,
                                "total_tokens": ev.prompt_tokens + ev.completion_tokens}, separators=(",", ":"))
            reason = "length" if ev.finish_reason == "length" else "stop"
            sink.finish(f'{base}"{reason}"{fin_body}{usage}}}\n\ndata: [DONE]\n\n'.encode())
        metrics.requests.labels(mid_, kind).inc()
        metrics.out_tokens.labels(mid_).inc(ev.completion_tokens)
        metrics.prompt_tokens.labels(mid_).inc(ev.prompt_tokens)
        tt = sink.ttft
        if tt >= 0:
            metrics.ttft.labels(mid_).observe(tt)
            if ev.completion_tokens > 1:
                metrics.itl.labels(mid_).observe((time.perf_counter() - t0 - tt) / (ev.completion_tokens - 1))
        if rep is not None:
            lm.handle._done(rep)
        loop.call_soon_threadsafe(state.manager.mark_busy, mid_, False)

    eng.add_request(prompt, params, on_final, sink=sink)
    return NativeHandledResponse()


async def handle_question(state, cfg, req, calls, result: str, prompt: str) -> str:
    """chat.go handleQuestion: answer from the no-action message, else re-run without grammar."""
    if not calls and result:
        return result
    args = calls[0].arguments if calls else ""
    try:
        a = json.loads(args) if args else {}
    except ValueError:
        a = {}
    msg = a.get("message") if isinstance(a, dict) else None
    if isinstance(msg, str) and msg:
        return finetune(cfg, prompt, msg)
    cfg.raw["grammar"] = ""
    text, _ = await Inference(state, cfg, req, "chat").predict(prompt)
    return finetune(cfg, prompt, text)


def _strip_trailing_zeros(v: List[float]) -> List[float]:
    """core/backend/embeddings.go:64-78."""
    i = len(v)
    while i > 0 and v[i - 1] == 0:
        i -= 1
    return v[:i]
