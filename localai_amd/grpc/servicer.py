"""Our native engine behind the `backend.Backend` contract.

Counterpart of the reference's C++ backend service (`backend/cpp/llama/grpc-server.cpp:
2304-2458` BackendServiceImpl): Health, LoadModel, Predict, PredictStream, Embedding,
TokenizeString, Status, GetMetrics, plus the in-memory vector store RPCs (the reference's
`local-store` Go backend, `backend/go/stores/store.go`, here on the GPU).  The same object is
used in-process by the gateway (the reference's unused `embedBackend` idea,
`pkg/grpc/embed.go`) or served over gRPC by `localai_amd.worker`.

Methods are asyncio coroutines with grpc.aio signatures `(request, context)`; `context`
may be None in-process.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import threading
import time
from typing import Optional

from . import backend_pb as pb
from ..utils import faults

log = logging.getLogger("localai_amd.servicer")


class Unimplemented(Exception):
    pass


class _Pump:
    """Moves engine-thread events onto the event loop with ONE loop wake-up per burst (the
    engine emits a whole decode step of events at once) instead of one per token."""

    def __init__(self, loop):
        import collections
        self.loop = loop
        self.dq = collections.deque()
        self.pending = False

    def push(self, ch, ev):
        self.dq.append((ch, ev))
        if not self.pending:
            self.pending = True
            self.loop.call_soon_threadsafe(self._drain)

    def _drain(self):
        self.pending = False
        dq = self.dq
        while dq:
            ch, ev = dq.popleft()
            ch._deliver(ev)


_PUMPS = {}


def _pump_for(loop) -> _Pump:
    p = _PUMPS.get(id(loop))
    if p is None or p.loop is not loop:
        p = _PUMPS[id(loop)] = _Pump(loop)
    return p


class _Channel:
    """Single-consumer event channel fed by a _Pump."""
    __slots__ = ("pump", "items", "waiter")

    def __init__(self, pump: _Pump):
        self.pump = pump
        self.items = []
        self.waiter = None

    def put(self, ev):  # engine thread
        self.pump.push(self, ev)

    def _deliver(self, ev):  # loop thread
        self.items.append(ev)
        w = self.waiter
        if w is not None and not w.done():
            w.set_result(None)

    async def get_all(self):
        while not self.items:
            self.waiter = self.pump.loop.create_future()
            await self.waiter
            self.waiter = None
        out, self.items = self.items, []
        return out


class EngineServicer:
    def __init__(self, device: Optional[str] = None, tp=None):
        self.engine = None
        self.device = device
        self.tp = tp
        self.store = None
        self.state = pb.StatusResponse.UNINITIALIZED
        self._lock = threading.Lock()
        self.model_name = ""

    # ------------------------------------------------------------------ helpers
    async def _abort(self, context, code, msg):
        if context is not None:
            import grpc
            await context.abort(code, msg)
        raise RuntimeError(msg)

    # ------------------------------------------------------------------ RPCs
    async def Health(self, request, context=None):
        eng = getattr(self, "engine", None)
        if eng is not None and not getattr(eng, "healthy", True):
            return pb.Reply(message=f"unhealthy: {eng.fatal_error}".encode())
        return pb.Reply(message=b"OK")

    async def LoadModel(self, request, context=None):
        from ..engine.llm_engine import EngineConfig, LLMEngine
        path = request.ModelFile or request.Model
        from ..models.hf_checkpoint import is_hf_checkpoint
        if not (os.path.isfile(path) or is_hf_checkpoint(path)):
            return pb.Result(success=False, message=f"model file not found: {path}")
        if self.engine is not None and getattr(self, "loaded_path", "") == os.path.abspath(path):
            return pb.Result(success=True, message="Loaded")  # pre-loaded (tensor-parallel worker group)
        try:
            import torch
            dev = self.device
            if dev is None:
                if torch.cuda.is_available():
                    idx = int(request.MainGPU) if request.MainGPU.isdigit() else 0
                    dev = f"cuda:{idx}"
                else:
                    dev = "cpu"
            ctx = request.ContextSize or 2048
            if request.MaxModelLen:
                ctx = request.MaxModelLen
            from ..models.whisper import WhisperModel, is_whisper_ggml
            if is_whisper_ggml(path):
                # whisper.cpp GGML speech model (the reference's whisper backend)
                loop = asyncio.get_running_loop()
                wm = await loop.run_in_executor(None, lambda: WhisperModel(path, dev))
                with self._lock:
                    self.engine, self.loaded_path = wm, os.path.abspath(path)
                    self.model_name = os.path.basename(path)
                    self.state = pb.StatusResponse.READY
                return pb.Result(success=True, message="Loaded")
            from ..gguf import GGUFReader
            from ..models.hf_checkpoint import hf_architecture
            from ..models.ggml_legacy import is_ggjt
            arch = (hf_architecture(path) if not os.path.isfile(path) else "llama" if is_ggjt(path)
                    else GGUFReader(path).architecture)
            if arch in ("bert", "nomic-bert"):
                # sentence-embedding encoder (bert-embeddings / sentencetransformers backends)
                from ..models.bert import BertConfig, BertEmbedder
                loop = asyncio.get_running_loop()
                emb = await loop.run_in_executor(None, lambda: BertEmbedder(BertConfig(path, dev, ctx)))
                with self._lock:
                    self.engine, self.loaded_path = emb, os.path.abspath(path)
                    self.model_name = os.path.basename(path)
                    self.state = pb.StatusResponse.READY
                return pb.Result(success=True, message="Loaded")
            cfg = EngineConfig(
                model_path=path, device=dev, context_size=ctx,
                max_num_seqs=int(os.environ.get("LOCALAI_MAX_NUM_SEQS", os.environ.get("LLAMACPP_PARALLEL", "256")) or 256),
                max_batched_tokens=max(int(request.NBatch or 0), 8192),
                gpu_memory_utilization=request.GPUMemoryUtilization or 0.85,
                embeddings=request.Embeddings, rope_freq_base=request.RopeFreqBase,
                rope_freq_scale=request.RopeFreqScale, rope_scaling=request.RopeScaling,
                use_graphs=not request.EnforceEager,
                mmproj=self._mmproj_path(request, path),
                lora_adapters=self._lora(request, path),
                draft_model=self._draft_path(request, path),
                quantization=str(request.Quantization or "") if is_hf_checkpoint(path) else "")
            loop = asyncio.get_running_loop()
            eng = await loop.run_in_executor(None, lambda: LLMEngine(cfg, tp=self.tp))
            await loop.run_in_executor(None, eng.warmup)
            eng.start()
            with self._lock:
                if self.engine is not None:
                    self.engine.shutdown()
                self.engine = eng
                self.loaded_path = os.path.abspath(path)
                self.model_name = os.path.basename(path)
                self.state = pb.StatusResponse.READY
            return pb.Result(success=True, message="Loaded")
        except Exception as e:  # report, do not crash the worker
            log.exception("LoadModel failed")
            self.state = pb.StatusResponse.ERROR
            return pb.Result(success=False, message=f"could not load model: {e}")

    @staticmethod
    def _lora(request, model_path: str):
        """grpc-server.cpp:2263-2271: an adapter only when both LoraAdapter and LoraBase are set,
        relative to the model's directory, scale LoraScale (1.0 when 0)."""
        if not request.LoraAdapter or not request.LoraBase:
            return ()
        from ..models.lora import adapter_path
        return ((adapter_path(model_path, request.LoraAdapter), float(request.LoraScale or 1.0)),)

    @staticmethod
    def _draft_path(request, model_path: str) -> str:
        """DraftModel, relative to the main model's directory (reference llama.go:89-95)."""
        d = str(request.DraftModel or "")
        if not d:
            return ""
        if not os.path.isabs(d):
            d = os.path.join(os.path.dirname(model_path), d)
        if not os.path.exists(d):
            raise FileNotFoundError(f"draft model {d} not found")
        return d

    @staticmethod
    def _mmproj_path(request, model_path: str) -> str:
        mm = request.MMProj
        if not mm:
            return ""
        return mm if os.path.isabs(mm) else os.path.join(os.path.dirname(model_path), mm)

    def _images(self, request):
        imgs = list(request.Images)
        if imgs and getattr(self.engine, "clip", None) is None:
            log.warning("request has %d image(s) but the model has no mmproj; ignoring them", len(imgs))
            return None
        return imgs or None

    def _require_engine(self):
        if self.engine is None:
            raise RuntimeError("no model loaded")
        return self.engine

    def _prompt(self, request):
        eng = self._require_engine()
        if request.UseTokenizerTemplate and len(request.Messages) and not request.Prompt:
            return self._apply_chat_template(request)
        return request.Prompt

    def _apply_chat_template(self, request) -> str:
        tok = self.engine.tokenizer
        msgs = [{"role": m.role, "content": m.content} for m in request.Messages]
        tpl = tok.chat_template
        if tpl:
            try:
                import jinja2
                env = jinja2.Environment(trim_blocks=True, lstrip_blocks=True)
                env.globals["raise_exception"] = lambda m: (_ for _ in ()).throw(ValueError(m))
                bos = tok.tokens[tok.bos_id] if tok.bos_id is not None and tok.bos_id >= 0 else ""
                eos = tok.tokens[tok.eos_id] if tok.eos_id is not None and tok.eos_id >= 0 else ""
                return env.from_string(tpl).render(messages=msgs, add_generation_prompt=True, bos_token=bos,
                                                   eos_token=eos)
            except Exception:
                log.exception("chat template failed; falling back to plain join")
        return "\n".join(f"{m['role']}: {m['content']}" for m in msgs) + "\nassistant:"

    def _params(self, request):
        from ..engine.sampling_params import SamplingParams
        return SamplingParams.from_predict_options(request)

    async def PredictStream(self, request, context=None):
        if os.environ.get("LOCALAI_AMD_WORKER") and faults.hit("worker_exit"):
            os._exit(17)  # injected fault: the worker process dies mid-service
        eng = self._require_engine()
        ch = _Channel(_pump_for(asyncio.get_running_loop()))
        rid = eng.add_request(self._prompt(request), self._params(request), ch.put, images=self._images(request))
        finished = False
        try:
            while True:
                evs = await ch.get_all()
                buf = bytearray()
                fin = None
                for ev in evs:  # coalesce everything already produced into one message
                    buf += ev.text
                    if ev.finished:
                        fin = ev
                        break
                if fin is not None:
                    finished = True
                    if fin.error:
                        raise RuntimeError(fin.error)
                    if buf:
                        yield pb.Reply(message=bytes(buf))
                    yield pb.Reply(message=b"", tokens=fin.completion_tokens, prompt_tokens=fin.prompt_tokens)
                    return
                if buf:
                    yield pb.Reply(message=bytes(buf))
                    if faults.hit("grpc_stream_drop"):
                        raise faults.InjectedFault("gRPC stream dropped (injected fault)")
        finally:
            if not finished:
                eng.abort(rid)  # client went away / generator closed: free the sequence (fixes Q4)

    async def Predict(self, request, context=None):
        eng = self._require_engine()
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        chunks = bytearray()

        def cb(ev):
            def apply():
                chunks.extend(ev.text)
                if ev.finished and not fut.done():
                    fut.set_result(ev)
            loop.call_soon_threadsafe(apply)

        rid = eng.add_request(self._prompt(request), self._params(request), cb, images=self._images(request))
        try:
            ev = await fut
        except asyncio.CancelledError:
            eng.abort(rid)
            raise
        if ev.error:
            await self._abort(context, _status("INTERNAL"), ev.error)  # fixes Q9 (error => gRPC error)
        return pb.Reply(message=bytes(chunks), tokens=ev.completion_tokens, prompt_tokens=ev.prompt_tokens)

    async def Embedding(self, request, context=None):
        eng = self._require_engine()
        loop = asyncio.get_running_loop()
        inp = list(request.EmbeddingTokens) if len(request.EmbeddingTokens) else (request.Embeddings or request.Prompt)
        vecs = await loop.run_in_executor(None, lambda: eng.embed([inp]))
        return pb.EmbeddingResult(embeddings=vecs[0])

    async def TokenizeString(self, request, context=None):
        eng = self._require_engine()
        toks = eng.tokenize(self._prompt(request))
        return pb.TokenizationResponse(length=len(toks), tokens=toks)

    async def Status(self, request, context=None):
        st = pb.StatusResponse(state=self.state)
        if self.engine is not None and self.engine.busy:
            st.state = pb.StatusResponse.BUSY
        try:
            import psutil
            rss = psutil.Process().memory_info().rss
            st.memory.breakdown["host_rss"] = rss
            total = rss
            import torch
            if self.engine is not None and self.engine.device.type == "cuda":
                free, tot = torch.cuda.mem_get_info(self.engine.device)
                st.memory.breakdown["gpu_used"] = tot - free
                st.memory.breakdown["gpu_total"] = tot
                st.memory.breakdown["kv_blocks_free"] = self.engine.sched.blocks().num_free
                total += tot - free
            st.memory.total = total
        except Exception:
            pass
        return st

    async def GetMetrics(self, request, context=None):
        """Metrics of the ACTIVE slot, as the reference's llama backend reports them
        (grpc-server.cpp:2434-2457): an in-flight request's id, prompt, generated tokens and
        decode rate; all zero / empty when nothing is in flight."""
        r = pb.MetricsResponse()
        s = None
        if self.engine is not None and hasattr(self.engine, "active_slot_stats"):
            s = self.engine.active_slot_stats()
        if s:
            r.slot_id = int(s["id"])
            r.tokens_per_second = float(s["tokens_per_second"])
            r.tokens_generated = int(s["completion_tokens"])
            r.prompt_tokens_processed = int(s["prompt_tokens"])
            # the slot's prompt as a JSON string (grpc-server.cpp:2441: slot->prompt.dump())
            r.prompt_json_for_slot = json.dumps(s["prompt"])
        return r

    # ------------------------------------------------------------------ vector store (local-store backend)
    def _store(self):
        if self.store is None:
            from ..engine.stores import VectorStore
            self.store = VectorStore(self.device)
        return self.store

    async def StoresSet(self, request, context=None):
        try:
            self._store().set([list(k.Floats) for k in request.Keys], [v.Bytes for v in request.Values])
            return pb.Result(success=True)
        except Exception as e:
            return pb.Result(success=False, message=str(e))

    async def StoresDelete(self, request, context=None):
        try:
            self._store().delete([list(k.Floats) for k in request.Keys])
            return pb.Result(success=True)
        except Exception as e:
            return pb.Result(success=False, message=str(e))

    async def StoresGet(self, request, context=None):
        keys, vals = self._store().get([list(k.Floats) for k in request.Keys])
        r = pb.StoresGetResult()
        for k, v in zip(keys, vals):
            r.Keys.add(Floats=k)
            r.Values.add(Bytes=v)
        return r

    async def StoresFind(self, request, context=None):
        keys, vals, sims = self._store().find(list(request.Key.Floats), request.TopK)
        r = pb.StoresFindResult(Similarities=sims)
        for k, v in zip(keys, vals):
            r.Keys.add(Floats=k)
            r.Values.add(Bytes=v)
        return r

    async def Rerank(self, request, context=None):
        """Jina rerank (reference `backend/python/rerankers/backend.py:60-95`).  A cross-encoder
        GGUF (BERT with a RANK head) scores each (query, doc) pair; any other model falls back to
        the cosine of its pooled embeddings (bi-encoder ranking)."""
        eng = self._require_engine()
        loop = asyncio.get_running_loop()
        docs = list(request.documents)
        scored = []
        if getattr(eng, "is_ranker", False):
            rel = await loop.run_in_executor(None, lambda: eng.rerank(request.query, docs))
            scored = [(s, i) for i, s in enumerate(rel)]
        else:
            vecs = await loop.run_in_executor(None, lambda: eng.embed([request.query] + docs))
            import math
            q = vecs[0]
            qn = math.sqrt(sum(x * x for x in q)) or 1.0
            for i, v in enumerate(vecs[1:]):
                vn = math.sqrt(sum(x * x for x in v)) or 1.0
                scored.append((sum(a * b for a, b in zip(q, v)) / (qn * vn), i))
        scored.sort(reverse=True)
        top = request.top_n if request.top_n > 0 else len(scored)
        res = pb.RerankResult()
        ntok = sum(len(d.split()) for d in docs) + len(request.query.split())
        res.usage.total_tokens = ntok
        res.usage.prompt_tokens = ntok
        for s, i in scored[:top]:
            res.results.add(index=i, text=docs[i], relevance_score=float(s))
        return res

    async def GenerateImage(self, request, context=None):
        raise Unimplemented("GenerateImage")

    async def TTS(self, request, context=None):
        raise Unimplemented("TTS")

    async def SoundGeneration(self, request, context=None):
        raise Unimplemented("SoundGeneration")

    async def AudioTranscription(self, request, context=None):
        """backend/go/transcribe/whisper/whisper.go:27-104: audio -> 16 kHz mono -> segments + text."""
        from ..models.whisper import WhisperModel, load_audio
        if not isinstance(self.engine, WhisperModel):
            raise Unimplemented("AudioTranscription (the loaded model is not a whisper model)")
        wm = self.engine

        def run():
            audio = load_audio(request.dst)
            return wm.transcribe(audio, language=request.language, translate=bool(request.translate))
        segs, text = await asyncio.get_running_loop().run_in_executor(None, run)
        return pb.TranscriptResult(
            segments=[pb.TranscriptSegment(id=s.id, start=s.start_ns, end=s.end_ns, text=s.text, tokens=s.tokens)
                      for s in segs], text=text)

    def shutdown(self):
        if self.engine is not None:
            self.engine.shutdown()
            self.engine = None


def _status(name):
    import grpc
    return getattr(grpc.StatusCode, name)
