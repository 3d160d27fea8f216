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


class DraftModel:
    """A small draft LM (config `draft_model`, path relative to the main model's directory as in
    the reference's `llama.go:89-95`) that proposes k greedy tokens per sequence; the engine
    verifies them with the main model in one forward (LLMEngine._run_spec), so the output stays
    exactly the main model's greedy output.

    The draft model keeps its own paged KV cache.  Per request it remembers which tokens its cache
    holds (`_cached`); a draft call first feeds every sequence the tokens it has not seen (the
    accepted tokens of the last verify, or the whole prompt the first time) in ONE chunked-prefill
    forward over all sequences (split into chunks of at most `max_batched_tokens` tokens, like the
    main engine's chunked prefill: a first draft feeds the whole prompt), then k-1 batched
    single-token decode forwards.  Cache entries past the accepted prefix are simply overwritten
    by the next call (longest-common-prefix rule)."""

    def __init__(self, path: str, device, max_seqs: int, context_size: int, vocab_size: int,
                 block_size: int = 32, max_batched_tokens: int = 2048):
        import torch

        from ..models.decoder import DecoderModel
        from ..models.hf_checkpoint import open_model
        self.torch = torch
        self.device = torch.device(device)
        self.reader = open_model(path)
        self.model = DecoderModel(self.reader, self.device, max_pos=context_size)
        if self.model.hp.n_vocab != vocab_size:
            raise ValueError(f"draft model vocabulary {self.model.hp.n_vocab} != main model {vocab_size}")
        self.bs = block_size
        self.ctx = context_size
        self.max_tokens = max(1, int(max_batched_tokens))  # catch-up tokens per forward
        self.max_blocks = (context_size + block_size - 1) // block_size
        nblk = max(1, max_seqs) * self.max_blocks + 1
        self.kv = self.model.new_kv_cache(nblk, block_size)
        self._free = list(range(nblk - 1, -1, -1))
        self._pages: dict = {}     # request id -> [page, ...]
        self._cached: dict = {}    # request id -> token ids whose K/V the cache holds
        self.ws = None

    def release(self, rid: int) -> None:
        self._free.extend(self._pages.pop(rid, []))
        self._cached.pop(rid, None)

    def _ensure_pages(self, rid: int, n_tokens: int, keep=()) -> list:
        pages = self._pages.setdefault(rid, [])
        need = (n_tokens + self.bs - 1) // self.bs
        while len(pages) < need:
            if not self._free:
                # evict a request that is not drafting now (it re-feeds its tokens next time)
                victim = next((r for r in self._pages if r != rid and r not in keep), None)
                if victim is None:
                    raise RuntimeError("draft model KV cache exhausted")
                self.release(victim)
                continue
            pages.append(self._free.pop())
        return pages

    def _slot(self, pages, p: int) -> int:
        return pages[p // self.bs] * self.bs + p % self.bs

    def _i32(self, a):
        return self.torch.tensor(np.asarray(a, dtype=np.int32), device=self.device)

    def _table(self, rids):
        bt = np.zeros((len(rids), max(len(self._pages[r]) for r in rids)), dtype=np.int32)
        for i, r in enumerate(rids):
            bt[i, :len(self._pages[r])] = self._pages[r]
        return self._i32(bt)

    def draft(self, rids: Sequence[int], seqs: Sequence[Sequence[int]], ks: Sequence[int]) -> List[List[int]]:
        """Greedy drafts of ks[i] tokens continuing seqs[i] (request rids[i])."""
        from .. import ops
        from ..models.decoder import ForwardBatch
        torch = self.torch
        live = [i for i, k in enumerate(ks) if k > 0 and len(seqs[i]) + k <= self.ctx]
        out: List[List[int]] = [[] for _ in seqs]
        if not live:
            return out
        # 1) catch-up: tokens the draft cache has not seen, as chunked-prefill forwards of at most
        #    max_tokens tokens (a sequence's range may span several chunks, in position order)
        segs = []
        for i in live:
            rid, seq = rids[i], list(seqs[i])
            old = self._cached.get(rid, [])
            lcp = 0
            m = min(len(old), len(seq) - 1)  # always re-feed at least the last token
            while lcp < m and old[lcp] == seq[lcp]:
                lcp += 1
            self._ensure_pages(rid, len(seq) + ks[i], keep=set(rids))
            segs.append((i, lcp, len(seq)))
            self._cached[rid] = seq
        chunks, cur, n = [], [], 0
        for i, a, b in segs:
            while a < b:
                take = min(b - a, self.max_tokens - n)
                cur.append((i, a, a + take))
                n += take
                a += take
                if n >= self.max_tokens:
                    chunks.append(cur)
                    cur, n = [], 0
        if cur:
            chunks.append(cur)
        for ch in chunks:
            toks, pos, slots, cu, ctxl = [], [], [], [0], []
            for i, a, b in ch:
                seq, pages = seqs[i], self._pages[rids[i]]
                for p in range(a, b):
                    toks.append(seq[p])
                    pos.append(p)
                    slots.append(self._slot(pages, p))
                cu.append(len(toks))
                ctxl.append(b)
            qlens = [cu[j + 1] - cu[j] for j in range(len(ch))]
            fb = ForwardBatch(tokens=self._i32(toks), pos=self._i32(pos), slots=self._i32(slots), decode=False,
                              block_tables=self._table([rids[i] for i, _, _ in ch]), cu_q=self._i32(cu),
                              ctx_lens=self._i32(ctxl),
                              tiles=ops.prefill_tiles(qlens, self.device) if self.device.type == "cuda" else None,
                              logits_idx=self._i32([c - 1 for c in cu[1:]]))
            nxt = self.model.forward(fb, self.kv).argmax(-1).tolist()
            for j, (i, a, b) in enumerate(ch):
                if b == len(seqs[i]):     # the piece holding the sequence's last token
                    out[i].append(int(nxt[j]))
        # 2) k-1 batched single-token decode forwards over the sequences still drafting
        kmax = max(ks[i] for i in live)
        for step in range(1, kmax):
            act = [j for j, i in enumerate(live) if ks[i] > step]
            if not act:
                break
            ids = [live[j] for j in act]
            tk = [out[i][-1] for i in ids]
            ps = [len(seqs[i]) + step - 1 for i in ids]
            sl = [self._slot(self._pages[rids[i]], p) for i, p in zip(ids, ps)]
            lens = [p + 1 for p in ps]
            fb = ForwardBatch(tokens=self._i32(tk), pos=self._i32(ps), slots=self._i32(sl), decode=True,
                              block_tables=self._table([rids[i] for i in ids]), seq_lens=self._i32(lens),
                              max_len=max(lens))
            am = self.model.forward(fb, self.kv, attn_workspace=self._workspace(len(ids))).argmax(-1).tolist()
            for i, t, p in zip(ids, am, ps):
                out[i].append(int(t))
                self._cached[rids[i]] = self._cached[rids[i]] + [out[i][-2]]  # K/V of p now cached
        return out

    def _workspace(self, B: int):
        if self.device.type != "cuda":
            return None
        from .. import ops
        if self.ws is None or self.ws[0] < B:
            hp = self.model
            self.ws = (B, ops.decode_workspace(B, hp.Hq, hp.Hkv, hp.Dh, self.ctx, self.device, self.bs))
        return self.ws[1]
