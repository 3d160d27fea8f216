"""Persistent prompt cache (`prompt_cache_path` / `prompt_cache_all` / `prompt_cache_ro`).

Reference: the model-config keys reach the backend as PredictOptions.PromptCachePath (joined
with the models directory), PromptCacheAll and PromptCacheRO (`core/backend/options.go:181-190`).
Only the legacy go-llama backend honours them (`backend/go/llm/llama/llama.go:131-142`: a
llama.cpp session file); the C++ server keeps prefix reuse in memory only.

Here the engine already has a global hashed prefix cache over paged KV blocks; the file simply
persists the FULL KV blocks of a prompt so the prefix cache can be warmed after a restart:

* save (at request finish, unless read-only): the token ids of the prompt (or prompt +
  generated tokens with prompt_cache_all) rounded down to whole KV blocks, and for every layer
  those blocks' K and V pages (bf16), in a safetensors file -- nothing executable, read back
  with the safetensors reader only.  Shape metadata guards against another model's cache.
* load (when a request names the file, once per file modification): the blocks are written into
  free KV blocks and registered in the prefix-cache hash chain exactly as if a request had just
  computed them, then released to the LRU; the request itself (and every later one sharing the
  prefix) then reuses them through the ordinary prefix lookup.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List

import torch

log = logging.getLogger("localai_amd.prompt_cache")

_FORMAT = "localai_amd.kvprefix.v1"


def _meta(engine) -> Dict[str, str]:
    m = engine.model
    return {"format": _FORMAT, "n_layer": str(engine.hp.n_layer), "n_kv": str(m.Hkv), "head_dim": str(m.Dh),
            "block_size": str(engine.kv.block_size), "model": os.path.basename(engine.cfg.model_path)}


def save(engine, sid: int, tokens: List[int], path: str) -> int:
    """Persist the KV of sequence `sid` for `tokens` (whole blocks).  Returns tokens saved."""
    from safetensors.torch import save_file
    bs = engine.kv.block_size
    nb = len(tokens) // bs
    if nb == 0:
        return 0
    table = engine.sched.blocks().table(sid)[:nb]
    idx = torch.tensor(table, dtype=torch.long, device=engine.kv.k[0].device)
    tensors = {"tokens": torch.tensor(tokens[:nb * bs], dtype=torch.int32)}
    for i in range(engine.hp.n_layer):
        tensors[f"k.{i}"] = engine.kv.k[i].index_select(0, idx).cpu().contiguous()
        tensors[f"v.{i}"] = engine.kv.v[i].index_select(0, idx).cpu().contiguous()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.partial{os.getpid()}"
    save_file(tensors, tmp, metadata=_meta(engine))
    os.replace(tmp, path)
    return nb * bs


def load(engine, path: str, scratch_sid: int) -> int:
    """Warm the prefix cache from `path`.  Returns the number of tokens made available."""
    from safetensors import safe_open
    with safe_open(path, framework="pt", device="cpu") as f:
        meta = f.metadata() or {}
        want = _meta(engine)
        for k in ("format", "n_layer", "n_kv", "head_dim", "block_size"):
            if meta.get(k) != want[k]:
                raise ValueError(f"prompt cache {path} does not match this model ({k}: {meta.get(k)} != {want[k]})")
        toks = f.get_tensor("tokens").tolist()
        bs = engine.kv.block_size
        nb = len(toks) // bs
        if nb == 0:
            return 0
        bm = engine.sched.blocks()
        # one extra token so every saved block counts as a full prefix block (the block manager
        # never reuses the block that holds a sequence's last token)
        cached = bm.allocate(scratch_sid, toks + [0], len(toks) + 1)
        if cached < 0:
            raise RuntimeError("not enough free KV blocks to restore it")
        try:
            table = bm.table(scratch_sid)
            first = cached // bs  # blocks already resident need no copy
            if first < nb:
                idx = torch.tensor(table[first:nb], dtype=torch.long, device=engine.kv.k[0].device)
                for i in range(engine.hp.n_layer):
                    k = f.get_tensor(f"k.{i}")[first:nb].to(engine.kv.k[i].device, engine.kv.k[i].dtype)
                    v = f.get_tensor(f"v.{i}")[first:nb].to(engine.kv.v[i].device, engine.kv.v[i].dtype)
                    engine.kv.k[i].index_copy_(0, idx, k)
                    engine.kv.v[i].index_copy_(0, idx, v)
            bm.commit(scratch_sid, toks, nb * bs)  # registers the hash chain
        finally:
            bm.free_seq(scratch_sid)  # blocks stay cached in the LRU
    return nb * bs


class PromptCacheFiles:
    """Per-engine bookkeeping: which cache files are resident (by modification time)."""

    def __init__(self):
        self._loaded: Dict[str, float] = {}
        self._scratch = -(1 << 40)

    def ensure_loaded(self, engine, path: str) -> int:
        try:
            mt = os.path.getmtime(path)
        except OSError:
            return 0
        if self._loaded.get(path) == mt:
            return 0
        self._scratch -= 1
        try:
            n = load(engine, path, self._scratch)
        except Exception as e:  # a stale / foreign / truncated file must not fail the request
            log.warning("prompt cache %s not loaded: %s", path, e)
            n = 0
        self._loaded[path] = mt
        return n

    def store(self, engine, sid: int, tokens: List[int], path: str) -> int:
        n = save(engine, sid, tokens, path)
        try:
            self._loaded[path] = os.path.getmtime(path)  # our own KV is already resident
        except OSError:
            pass
        return n
