"""`huggingface` backend (alias `langchain-huggingface`): text generation by the remote Hugging Face
Inference API, for models that are not served locally.

Reference: `backend/go/llm/langchain/langchain.go:14-64` (Load needs HUGGINGFACEHUB_API_TOKEN;
Predict / PredictStream forward model, max tokens, temperature and stop words; the stream sends
the whole completion as one message), `pkg/langchain/huggingface.go:13-58`, backend name
`pkg/model/initializers.go:28,54`.

The request is the Inference API's text-generation call: POST `<endpoint>/models/<repo id>` with
`{"inputs": prompt, "parameters": {...}, "options": {"wait_for_model": true}}` and a bearer
token; the reply is `[{"generated_text": ...}]`.  `return_full_text` is false so the completion
does not repeat the prompt (the upstream client's exact body is parity-unpinned).  The endpoint
defaults to https://api-inference.huggingface.co and can be pointed elsewhere (a TGI server, a
test double) with HF_INFERENCE_ENDPOINT.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

from . import backend_pb as pb

DEFAULT_ENDPOINT = "https://api-inference.huggingface.co"


class HuggingFaceServicer:
    """backend.proto servicer (Health, LoadModel, Predict, PredictStream, Status)."""

    def __init__(self):
        self.model = ""
        self.token = ""
        self.state = pb.StatusResponse.UNINITIALIZED

    async def Health(self, request, context):
        return pb.Reply(message=b"OK")

    async def LoadModel(self, request, context):
        token = os.environ.get("HUGGINGFACEHUB_API_TOKEN", "")
        if not token:
            return pb.Result(success=False, message="no huggingface token provided")
        self.token, self.model = token, request.Model
        self.state = pb.StatusResponse.READY
        return pb.Result(success=True, message="")

    async def Status(self, request, context):
        return pb.StatusResponse(state=self.state)

    def shutdown(self):
        self.token, self.state = "", pb.StatusResponse.UNINITIALIZED

    def _body(self, req) -> dict:
        params = {"temperature": float(req.Temperature), "return_full_text": False}
        if req.Tokens > 0:
            params["max_new_tokens"] = int(req.Tokens)
        if req.TopP > 0:
            params["top_p"] = float(req.TopP)
        if req.TopK > 0:
            params["top_k"] = int(req.TopK)
        stops: List[str] = [s for s in req.StopPrompts if s]
        if stops:
            params["stop"] = stops
        return {"inputs": req.Prompt, "parameters": params, "options": {"wait_for_model": True}}

    async def _call(self, req) -> str:
        import aiohttp
        if not self.token:
            raise RuntimeError("huggingface backend: model not loaded (no token)")
        url = f"{os.environ.get('HF_INFERENCE_ENDPOINT', DEFAULT_ENDPOINT).rstrip('/')}/models/{self.model}"
        headers = {"Authorization": f"Bearer {self.token}", "Content-Type": "application/json"}
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=600)) as s:
            async with s.post(url, data=json.dumps(self._body(req)), headers=headers) as r:
                raw = await r.read()
                if r.status != 200:
                    raise RuntimeError(f"huggingface inference API {r.status}: {raw[:300].decode('utf-8', 'replace')}")
        doc = json.loads(raw)
        if isinstance(doc, list) and doc and isinstance(doc[0], dict):
            return str(doc[0].get("generated_text", ""))
        if isinstance(doc, dict) and "generated_text" in doc:
            return str(doc["generated_text"])
        raise RuntimeError(f"huggingface inference API: unexpected reply {str(doc)[:200]}")

    @staticmethod
    def _cut_stops(text: str, stops) -> str:
        """The API may keep the stop sequence in the text; the completion ends before it."""
        cut: Optional[int] = None
        for s in stops:
            if s:
                i = text.find(s)
                if i >= 0 and (cut is None or i < cut):
                    cut = i
        return text if cut is None else text[:cut]

    async def Predict(self, request, context):
        text = self._cut_stops(await self._call(request), request.StopPrompts)
        return pb.Reply(message=text.encode("utf-8"))

    async def PredictStream(self, request, context):
        # langchain.go:52-63: one message with the whole completion, then the stream ends
        text = self._cut_stops(await self._call(request), request.StopPrompts)
        yield pb.Reply(message=text.encode("utf-8"))
