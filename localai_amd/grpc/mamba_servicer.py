"""`mamba` and `rwkv` backend servicers (backend.proto) over the recurrent models
(models/mamba.py, models/rwkv.py).

Mamba mirrors `backend/python/mamba/backend.py`: one request at a time (the reference runs one
gRPC worker), `Tokens == 0` -> 2000 new tokens, `TopP == 0` -> 0.9, generation stops at the eos
token.  RWKV mirrors `backend/go/llm/rwkv/rwkv.go`: stop word "\n" unless the request names stop
words, tokenizer file from `tokenizer` or `<model>.tokenizer.json`, TokenizeString.  Stop strings
are honoured with UTF-8 / partial-stop hold-back, and the final streamed Reply carries the token
counts like the engine's streams.
"""
from __future__ import annotations

import asyncio
import os
import threading
from typing import Iterator, List, Tuple

from . import backend_pb as pb


class MambaServicer:
    DEFAULT_STOPS: List[str] = []

    def __init__(self, device: str = ""):
        self.device = device
        self.model = None
        self.state = pb.StatusResponse.UNINITIALIZED
        self._lock = threading.Lock()

    async def Health(self, request, context):
        return pb.Reply(message=b"OK")

    async def Status(self, request, context):
        return pb.StatusResponse(state=self.state)

    def _check(self, path: str) -> bool:
        from ..models.mamba import is_mamba_checkpoint
        return is_mamba_checkpoint(path)

    def _build(self, path: str, dev: str, request):
        from ..models.mamba import MambaLM
        return MambaLM(path, dev)

    async def LoadModel(self, request, context):
        path = request.ModelFile or request.Model
        if not self._check(path):
            return pb.Result(success=False, message=f"not a {type(self).__name__[:-9]} checkpoint: {path}")
        dev = self.device
        if not dev:
            import torch
            dev = "cuda:0" if torch.cuda.is_available() else "cpu"
        try:
            m = await asyncio.get_running_loop().run_in_executor(None, lambda: self._build(path, dev, request))
        except Exception as e:  # noqa: BLE001 - reported to the caller like the reference
            return pb.Result(success=False, message=f"Unexpected {e!r}")
        self.model, self.state = m, pb.StatusResponse.READY
        return pb.Result(success=True, message="Model loaded successfully")

    def shutdown(self):
        self.model, self.state = None, pb.StatusResponse.UNINITIALIZED

    async def TokenizeString(self, request, context):
        ids = self._require().tokenize(request.Prompt)
        return pb.TokenizationResponse(length=len(ids), tokens=ids)

    def _require(self):
        if self.model is None:
            raise RuntimeError("no model loaded")
        return self.model

    def _generate(self, request) -> Iterator[Tuple[str, int, int]]:
        """Yields (text delta, prompt tokens, generated tokens)."""
        import torch

        from ..models.mamba import sample
        m = self._require()
        max_new = request.Tokens if request.Tokens > 0 else 2000
        top_p = request.TopP if request.TopP > 0 else 0.9
        gen = torch.Generator().manual_seed(request.Seed if request.Seed > 0 else int.from_bytes(os.urandom(4), "little"))
        stops: List[str] = [s for s in request.StopPrompts if s] or list(self.DEFAULT_STOPS)
        ids = m.tokenize(request.Prompt)
        st = m.new_state(1)
        logits = m.prefill(ids, st)[-1]
        out: List[int] = []
        emitted = ""
        for _ in range(max_new):
            t = sample(logits, request.Temperature, top_p, request.TopK, gen)
            if m.eos_id is not None and t == m.eos_id:
                break
            out.append(t)
            text = m.decode(out)
            cut = min((text.find(s) for s in stops if s in text), default=-1)
            if cut >= 0:
                if cut > len(emitted):
                    yield text[len(emitted):cut], len(ids), len(out)
                return
            # hold back an incomplete UTF-8 sequence and any suffix that may start a stop string
            safe = len(text) - (1 if text.endswith("�") else 0)
            for s in stops:
                for k in range(min(len(s) - 1, safe), 0, -1):
                    if text[:safe].endswith(s[:k]):
                        safe -= k
                        break
            if safe > len(emitted):
                yield text[len(emitted):safe], len(ids), len(out)
                emitted = text[:safe]
            logits = m.step(torch.tensor([t], device=m.device), st)[0]
        text = m.decode(out)
        if len(text) > len(emitted):
            yield text[len(emitted):], len(ids), len(out)
        else:
            yield "", len(ids), len(out)

    def _run(self, request) -> List[Tuple[str, int, int]]:
        with self._lock:
            return list(self._generate(request))

    async def Predict(self, request, context):
        parts = await asyncio.get_running_loop().run_in_executor(None, self._run, request)
        text = "".join(p[0] for p in parts)
        n_prompt, n_gen = (parts[-1][1], parts[-1][2]) if parts else (0, 0)
        return pb.Reply(message=text.encode("utf-8"), tokens=n_gen, prompt_tokens=n_prompt)

    async def PredictStream(self, request, context):
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()

        def work():
            try:
                with self._lock:
                    for part in self._generate(request):
                        loop.call_soon_threadsafe(q.put_nowait, part)
            except Exception as e:  # noqa: BLE001
                loop.call_soon_threadsafe(q.put_nowait, e)
            loop.call_soon_threadsafe(q.put_nowait, None)
        threading.Thread(target=work, daemon=True).start()
        last = (0, 0)
        while True:
            item = await q.get()
            if item is None:
                break
            if isinstance(item, Exception):
                raise item
            text, n_prompt, n_gen = item
            last = (n_prompt, n_gen)
            if text:
                yield pb.Reply(message=text.encode("utf-8"))
        yield pb.Reply(message=b"", tokens=last[1], prompt_tokens=last[0])


class RwkvServicer(MambaServicer):
    DEFAULT_STOPS = ["\n"]  # rwkv.go:41-44

    def _check(self, path: str) -> bool:
        from ..models.rwkv import is_rwkv_checkpoint
        return is_rwkv_checkpoint(path)

    def _build(self, path: str, dev: str, request):
        from ..models.rwkv import RwkvLM
        return RwkvLM(path, dev, request.Tokenizer)
