"""Per-request generation parameters (the PredictOptions sampling surface,
`backend/backend.proto:106-153`, as consumed by `grpc-server.cpp:2068-2134`)."""
from __future__ import annotations

import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class SamplingParams:
    max_tokens: int = -1              # <= 0: until EOS / context full
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.95
    min_p: float = 0.05               # llama.cpp default (not exposed by the proto)
    typical_p: float = 1.0
    tfs_z: float = 1.0
    repeat_penalty: float = 1.0
    repeat_last_n: int = 64
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    penalize_nl: bool = False
    mirostat: int = 0
    mirostat_tau: float = 5.0
    mirostat_eta: float = 0.1
    seed: int = -1
    ignore_eos: bool = False
    stop: List[str] = field(default_factory=list)
    logit_bias: Dict[int, float] = field(default_factory=dict)
    n_keep: int = 0
    grammar: str = ""
    n_probs: int = 0
    correlation_id: str = ""          # X-Correlation-ID of the HTTP request (PredictOptions.CorrelationId)
    n_draft: int = 0                  # speculative (n-gram) draft length for greedy requests
    prompt_cache_path: str = ""       # persistent KV prefix file (engine/prompt_cache.py)
    prompt_cache_all: bool = False    # also persist the generated tokens' KV
    prompt_cache_ro: bool = False     # read the file, never write it

    def resolved_seed(self) -> int:
        if self.seed is None or self.seed < 0:
            self.seed = random.getrandbits(31)
        return self.seed

    @staticmethod
    def from_predict_options(po) -> "SamplingParams":
        """Map a backend.proto PredictOptions message (grpc-server.cpp parse_options)."""
        sp = SamplingParams(
            max_tokens=int(po.Tokens) if po.Tokens else -1,
            temperature=float(po.Temperature),
            top_k=int(po.TopK),
            top_p=float(po.TopP) if po.TopP else 1.0,
            typical_p=float(po.TypicalP) if po.TypicalP else 1.0,
            tfs_z=float(po.TailFreeSamplingZ) if po.TailFreeSamplingZ else 1.0,
            repeat_penalty=float(po.Penalty) if po.Penalty else 1.0,
            repeat_last_n=int(po.Repeat),
            frequency_penalty=float(po.FrequencyPenalty),
            presence_penalty=float(po.PresencePenalty),
            penalize_nl=bool(po.PenalizeNL),
            mirostat=int(po.Mirostat),
            mirostat_tau=float(po.MirostatTAU) if po.MirostatTAU else 5.0,
            mirostat_eta=float(po.MirostatETA) if po.MirostatETA else 0.1,
            seed=int(po.Seed),
            ignore_eos=bool(po.IgnoreEOS),
            stop=[s for s in po.StopPrompts if s],
            n_keep=int(po.NKeep),
            grammar=po.Grammar,
            correlation_id=po.CorrelationId,
            n_draft=int(po.NDraft),
            prompt_cache_path=po.PromptCachePath,
            prompt_cache_all=bool(po.PromptCacheAll),
            prompt_cache_ro=bool(po.PromptCacheRO),
        )
        if po.LogitBias:
            import json
            try:
                lb = json.loads(po.LogitBias)
                sp.logit_bias = {int(k): float(v) for k, v in lb.items()}
            except Exception:
                pass
        return sp
