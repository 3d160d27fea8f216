"""Request orchestration: merge request into model config, build PredictOptions, run the
backend, post-process (`core/backend/{llm,options}.go`, `core/http/endpoints/openai/
{request,inference}.go`)."""
from __future__ import annotations

import base64
import json
import logging
import os
import re
import threading
import time
from dataclasses import dataclass
from typing import AsyncIterator, List, Optional, Tuple

from ..config.backend_config import BackendConfig
from ..grpc import backend_pb as pb
from ..templates import template_multimodal

log = logging.getLogger("localai_amd.inference")


@dataclass
class TokenUsage:
    prompt: int = 0
    completion: int = 0


# --------------------------------------------------------------------------- request -> config
def content_uri_as_base64(s: str) -> str:
    """utils.GetContentURIAsBase64: data: URIs or http(s) URLs -> base64 payload."""
    if s.startswith("data:"):
        return s.split(",", 1)[1] if "," in s else ""
    if s.startswith(("http://", "https://")):
        import urllib.request
        with urllib.request.urlopen(s, timeout=30) as r:  # noqa: S310 (user-requested fetch)
            return base64.b64encode(r.read()).decode()
    raise ValueError("not valid string")


def update_request_config(cfg: BackendConfig, req: dict):
    """updateRequestConfig (request.go:51-296): request fields override config fields."""
    P = cfg.raw["parameters"]
    if req.get("echo"):
        P["echo"] = True
    for k in ("top_k", "top_p", "temperature", "max_tokens", "seed", "typical_p"):
        if req.get(k) is not None:
            P[k] = req[k]
    if req.get("backend"):
        cfg.backend = req["backend"]
    if req.get("negative_prompt"):
        P["negative_prompt"] = req["negative_prompt"]
    if req.get("rope_freq_base"):
        P["rope_freq_base"] = req["rope_freq_base"]
    if req.get("rope_freq_scale"):
        P["rope_freq_scale"] = req["rope_freq_scale"]
    if req.get("grammar"):
        cfg.raw["grammar"] = req["grammar"]
    rf = req.get("response_format")
    if isinstance(rf, str):
        cfg.response_format = rf
    elif isinstance(rf, dict):
        cfg.response_format_map = rf
    stop = req.get("stop")
    sw = cfg.stopwords
    if isinstance(stop, str) and stop:
        sw.append(stop)
    elif isinstance(stop, list):
        sw.extend(s for s in stop if isinstance(s, str))
    cfg.stopwords = sw
    funcs = list(req.get("functions") or [])
    for t in req.get("tools") or []:
        if isinstance(t, dict) and t.get("function"):
            funcs.append(t["function"])
    req["_functions"] = funcs
    tc = req.get("tool_choice")
    if tc is not None:
        name = ""
        if isinstance(tc, str):
            try:
                name = ((json.loads(tc) or {}).get("function") or {}).get("name", "")
            except ValueError:
                name = ""
        elif isinstance(tc, dict):
            name = (tc.get("function") or {}).get("name", "")
        req["function_call"] = {"name": name}
    # decode multimodal message content into StringContent + placeholders
    img = vid = aud = 0
    tpl = cfg.template
    for m in req.get("messages") or []:
        c = m.get("content")
        m["_images"], m["_videos"], m["_audios"] = [], [], []
        if isinstance(c, str):
            m["_string_content"] = c
        elif isinstance(c, list):
            m["_string_content"] = ""
            for part in c:
                if not isinstance(part, dict):
                    continue
                t = part.get("type")
                if t == "text":
                    m["_string_content"] = part.get("text", "")
                elif t in ("image_url", "image"):
                    try:
                        b64 = content_uri_as_base64((part.get("image_url") or {}).get("url", ""))
                    except Exception:
                        continue
                    m["_images"].append(b64)
                    m["_string_content"] = template_multimodal(tpl.get("image") or "[img-{{.ID}}]{{.Text}}", img,
                                                               m["_string_content"])
                    img += 1
                elif t in ("video_url", "video"):
                    try:
                        b64 = content_uri_as_base64((part.get("video_url") or {}).get("url", ""))
                    except Exception:
                        continue
                    m["_videos"].append(b64)
                    m["_string_content"] = template_multimodal(tpl.get("video") or "[vid-{{.ID}}]{{.Text}}", vid,
                                                               m["_string_content"])
                    vid += 1
                elif t in ("audio_url", "audio"):
                    try:
                        b64 = content_uri_as_base64((part.get("audio_url") or {}).get("url", ""))
                    except Exception:
                        continue
                    m["_audios"].append(b64)
                    m["_string_content"] = template_multimodal(tpl.get("audio") or "[audio-{{.ID}}]{{.Text}}", aud,
                                                               m["_string_content"])
                    aud += 1
        else:
            m["_string_content"] = ""
    for k in ("repeat_penalty", "frequency_penalty", "presence_penalty", "batch", "repeat_last_n"):
        if req.get(k):
            P[k] = req[k]
    if req.get("n_keep"):
        P["n_keep"] = req["n_keep"]
    if req.get("ignore_eos"):
        P["ignore_eos"] = True
    # extension: allow disabling mirostat per request (config-level knob in the reference)
    if req.get("mirostat") is not None:
        cfg.raw["mirostat"] = req["mirostat"]
    inp = req.get("input")
    if isinstance(inp, str):
        if inp:
            cfg.input_strings.append(inp)
    elif isinstance(inp, list):
        for x in inp:
            if isinstance(x, str):
                cfg.input_strings.append(x)
            elif isinstance(x, list):
                cfg.input_tokens.append([int(t) for t in x])
            elif isinstance(x, (int, float)):
                # a flat list of token ids is one tokenized input
                cfg.input_tokens.append([int(t) for t in inp])
                break
    fc = req.get("function_call")
    if isinstance(fc, str):
        if fc:
            cfg.function_call_string = fc
    elif isinstance(fc, dict):
        cfg.function_call_name_string = str(fc.get("name") or "")
    pr = req.get("prompt")
    if isinstance(pr, str):
        cfg.prompt_strings.append(pr)
    elif isinstance(pr, list):
        cfg.prompt_strings.extend(p for p in pr if isinstance(p, str))


def predict_options(cfg: BackendConfig, prompt: str, messages: Optional[list] = None,
                    models_path: str = "") -> pb.PredictOptions:
    """gRPCPredictOpts (core/backend/options.go:180-229)."""
    P = cfg.raw["parameters"]
    r = cfg.raw
    pc_path = ""
    if r.get("prompt_cache_path"):  # options.go:181-190: relative to the models directory
        pc_path = os.path.join(models_path, str(r["prompt_cache_path"]))
        os.makedirs(os.path.dirname(pc_path) or ".", exist_ok=True)
    po = pb.PredictOptions(
        Prompt=prompt,
        Temperature=float(P.get("temperature") if P.get("temperature") is not None else 0.9),
        TopP=float(P.get("top_p") if P.get("top_p") is not None else 0.95),
        TopK=int(P.get("top_k") if P.get("top_k") is not None else 40),
        Tokens=int(P.get("max_tokens") or 0),
        Threads=int(r.get("threads") or 4),
        NDraft=int(r.get("n_draft") or 0),
        PromptCacheAll=bool(r.get("prompt_cache_all")), PromptCacheRO=bool(r.get("prompt_cache_ro")),
        PromptCachePath=pc_path,
        F16KV=bool(r.get("f16")), DebugMode=bool(r.get("debug")), Grammar=str(r.get("grammar") or ""),
        NegativePromptScale=float(P.get("negative_prompt_scale") or 0),
        RopeFreqBase=float(P.get("rope_freq_base") or 0), RopeFreqScale=float(P.get("rope_freq_scale") or 0),
        NegativePrompt=str(P.get("negative_prompt") or ""),
        Mirostat=int(r.get("mirostat") if r.get("mirostat") is not None else 2),
        MirostatETA=float(r.get("mirostat_eta") if r.get("mirostat_eta") is not None else 0.1),
        MirostatTAU=float(r.get("mirostat_tau") if r.get("mirostat_tau") is not None else 5.0),
        Debug=bool(r.get("debug")), StopPrompts=cfg.stopwords, Repeat=int(P.get("repeat_last_n") or 0),
        FrequencyPenalty=float(P.get("frequency_penalty") or 0), PresencePenalty=float(P.get("presence_penalty") or 0),
        Penalty=float(P.get("repeat_penalty") or 0), NKeep=int(P.get("n_keep") or 0), Batch=int(P.get("batch") or 0),
        IgnoreEOS=bool(P.get("ignore_eos")), Seed=cfg.resolved_seed() & 0x7FFFFFFF, MLock=bool(r.get("mmlock")),
        MMap=bool(r.get("mmap")), MainGPU=str(r.get("main_gpu") or ""), TensorSplit=str(r.get("tensor_split") or ""),
        TailFreeSamplingZ=float(P.get("tfz") if P.get("tfz") is not None else 1.0),
        TypicalP=float(P.get("typical_p") if P.get("typical_p") is not None else 1.0),
        UseTokenizerTemplate=bool(cfg.template.get("use_tokenizer_template")),
    )
    if messages and cfg.template.get("use_tokenizer_template") and not prompt:
        for m in messages:
            po.Messages.add(role=m.get("role", ""), content=m.get("_string_content", "") or str(m.get("content") or ""))
    return po


def finetune(cfg: BackendConfig, inp: str, prediction: str) -> str:
    """core/backend/llm.go:168-216 (echo, cutstrings, extract_regex, trimspace, trimsuffix)."""
    P = cfg.raw["parameters"]
    r = cfg.raw
    if P.get("echo"):
        prediction = inp + prediction
    for c in r.get("cutstrings") or []:
        prediction = re.sub(c, "", prediction)
    res = ""
    for rx in r.get("extract_regex") or []:
        m = re.search(rx, prediction)
        if m:
            res += m.group(0)
    if res:
        prediction = res
    for c in r.get("trimspace") or []:
        prediction = (prediction[len(c):] if c and prediction.startswith(c) else prediction).strip()
    for c in r.get("trimsuffix") or []:
        prediction = (prediction[:-len(c)] if c and prediction.endswith(c) else prediction).strip()
    return prediction


class Inference:
    """backend.ModelInference: stream or one-shot, with token usage."""

    def __init__(self, state, cfg: BackendConfig, req: dict, endpoint: str):
        self.state, self.cfg, self.req, self.endpoint = state, cfg, req, endpoint

    def _media(self, po):
        for m in self.req.get("messages") or []:
            po.Images.extend(m.get("_images", []))
            po.Videos.extend(m.get("_videos", []))
            po.Audios.extend(m.get("_audios", []))
        po.CorrelationId = self.req.get("_correlation_id", "")

    async def _backend(self):
        lm = await self.state.manager.load(self.cfg)
        return lm

    async def stream(self, prompt: str) -> AsyncIterator[Tuple[str, TokenUsage, bool]]:
        """Yields (text_delta, usage, is_final).  Text deltas are whole UTF-8 sequences."""
        lm = await self._backend()
        po = predict_options(self.cfg, prompt, self.req.get("messages"), self.state.models_path)
        self._media(po)
        mid = lm.id
        self.state.manager.mark_busy(mid, True)
        usage = TokenUsage()
        t0 = time.perf_counter()
        first = None
        pending = b""
        try:
            async for rep in lm.handle.PredictStream(po):
                if rep.tokens or rep.prompt_tokens:
                    usage.completion, usage.prompt = rep.tokens, rep.prompt_tokens
                data = pending + bytes(rep.message)
                if not data:
                    continue
                # keep incomplete UTF-8 tails for the next message (llm.go:123-138 rune loop)
                cut = len(data)
                for i in range(1, min(4, len(data)) + 1):
                    b = data[-i]
                    if b & 0xC0 == 0x80:
                        continue
                    need = 2 if b & 0xE0 == 0xC0 else 3 if b & 0xF0 == 0xE0 else 4 if b & 0xF8 == 0xF0 else 1
                    if need > i:
                        cut = len(data) - i
                    break
                pending = data[cut:]
                text = data[:cut].decode("utf-8", errors="replace")
                if text:
                    if first is None:
                        first = time.perf_counter()
                        self.state.metrics.ttft.labels(mid).observe(first - t0)
                    usage.completion = max(usage.completion, 0)
                    yield text, usage, False
            if pending:
                yield pending.decode("utf-8", errors="replace"), usage, False
            yield "", usage, True
        finally:
            self.state.manager.mark_busy(mid, False)
            self._account(mid, usage, t0, first)

    async def predict(self, prompt: str) -> Tuple[str, TokenUsage]:
        lm = await self._backend()
        po = predict_options(self.cfg, prompt, self.req.get("messages"), self.state.models_path)
        self._media(po)
        self.state.manager.mark_busy(lm.id, True)
        t0 = time.perf_counter()
        try:
            rep = await lm.handle.Predict(po)
        finally:
            self.state.manager.mark_busy(lm.id, False)
        usage = TokenUsage(rep.prompt_tokens, rep.tokens)
        if self.cfg.feature_enabled("usage") and not usage.prompt:
            try:
                tr = await lm.handle.TokenizeString(po)
                usage.prompt = tr.length
            except Exception:
                pass
        self._account(lm.id, usage, t0, None)
        return bytes(rep.message).decode("utf-8", errors="replace"), usage

    def _account(self, mid, usage, t0, first):
        m = self.state.metrics
        m.requests.labels(mid, self.endpoint).inc()
        m.out_tokens.labels(mid).inc(usage.completion)
        m.prompt_tokens.labels(mid).inc(usage.prompt)
        if first is not None and usage.completion > 1:
            m.itl.labels(mid).observe((time.perf_counter() - first) / (usage.completion - 1))
