"""Speculative decoding drafts (PredictOptions.NDraft, config `n_draft` / `draft_model`).

Reference: `n_draft` / `draft_model` reach the backends through the proto
(`backend/backend.proto:146,210`, `core/config/backend_config.go:143-144`); only the legacy
go-llama backend (unbuilt in the reference tree) implements them, with a draft model
(`backend/go/llm/llama/llama.go:82-101,202-204`).  SURVEY §2.10 "Speculative decoding: later
phase (draft model or n-gram)".

Ours is prompt-lookup (n-gram) speculation for greedy sequences: the draft is the continuation of
the most recent earlier occurrence of the sequence's last n tokens (n = 3, 2, 1).  The engine
verifies all drafted tokens of a batch in ONE forward pass (the chunked-prefill path: each
sequence feeds its last token + draft at positions L-1 .. L-1+k against its paged KV) and keeps
the longest prefix the model's own argmax agrees with plus the model's next token -- so the
output is exactly the greedy output, in fewer weight-streaming passes when drafts hit
(code, JSON, templated or repetitive text).  Rejected positions only leave KV past the
sequence end, which the next step overwrites.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def ngram_draft(seq: Sequence[int], k: int, max_n: int = 3, min_n: int = 1) -> List[int]:
    """Up to k tokens that followed the latest earlier match of seq's last n tokens."""
    L = len(seq)
    if k <= 0 or L < 2:
        return []
    a = np.asarray(seq, dtype=np.int64)
    for n in range(min(max_n, L - 1), min_n - 1, -1):
        pat = a[L - n:]
        win = np.lib.stride_tricks.sliding_window_view(a[:L - 1], n)  # starts 0 .. L-1-n
        hits = np.nonzero((win == pat).all(axis=1))[0]
        if len(hits):
            s = int(hits[-1]) + n
            d = a[s:s + k]
            if len(d):
                return d.tolist()
    return []
