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
import threading
from typing import Dict, List

import torch

log = logging.getLogger("localai_amd.prompt_cache")

_FORMAT = "localai_amd.kvprefix.v1"


def _meta(engine) -> Dict[str, str]:
    m = engine.model
    return {"format": _FORMAT, "n_layer": str(engine.hp.n_layer), "n_kv": str(m.Hkv), "head_dim": str(m.Dh),
            "block_size": str(engine.kv.block_size), "model": os.path.basename(engine.cfg.model_path)}


def snapshot(engine, sid: int, tokens: List[int]):
    """Gather the KV pages of sequence `sid` for `tokens` (whole blocks) into one host buffer.

    Runs on the engine thread: one index_select per layer into a device staging tensor (stream-
    ordered before any later reuse of those blocks), then ONE non-blocking copy into pinned host
    memory.  Returns (tokens, host tensor, event) or None; nothing here waits for the GPU."""
    bs = engine.kv.block_size
    nb = len(tokens) // bs
    if nb == 0:
        return None
    table = engine.sched.blocks().table(sid)[:nb]
    k0, v0 = engine.kv.k[0], engine.kv.v[0]  # V pages may be stored transposed: own buffer
    idx = torch.tensor(table, dtype=torch.long, device=k0.device)
    L = engine.hp.n_layer
    dk = torch.empty((L, nb) + tuple(k0.shape[1:]), dtype=k0.dtype, device=k0.device)
    dv = torch.empty((L, nb) + tuple(v0.shape[1:]), dtype=v0.dtype, device=v0.device)
    for i in range(L):
        torch.index_select(engine.kv.k[i], 0, idx, out=dk[i])
        torch.index_select(engine.kv.v[i], 0, idx, out=dv[i])
    if dk.is_cuda:
        hk = torch.empty(dk.shape, dtype=dk.dtype, pin_memory=True)
        hv = torch.empty(dv.shape, dtype=dv.dtype, pin_memory=True)
        hk.copy_(dk, non_blocking=True)
        hv.copy_(dv, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
    else:
        hk, hv, ev = dk, dv, None
    return list(tokens[:nb * bs]), (hk, hv), ev


def write(engine_meta: Dict[str, str], snap, path: str) -> int:
    """Write a snapshot as safetensors (background thread: waits for the copy, not the engine)."""
    from safetensors.torch import save_file
    toks, host, ev = snap
    if ev is not None:
        ev.synchronize()
    hk, hv = host
    tensors = {"tokens": torch.tensor(toks, dtype=torch.int32)}
    for i in range(hk.shape[0]):
        tensors[f"k.{i}"] = hk[i].contiguous()
        tensors[f"v.{i}"] = hv[i].contiguous()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.partial{os.getpid()}.{threading.get_ident()}"
    save_file(tensors, tmp, metadata=engine_meta)
    os.replace(tmp, path)
    return len(toks)


def save(engine, sid: int, tokens: List[int], path: str) -> int:
    """Synchronous save (tools / tests): snapshot + write."""
    snap = snapshot(engine, sid, tokens)
    return 0 if snap is None else write(_meta(engine), snap, path)


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
    """Per-engine bookkeeping: which cache files are resident (by modification time), which token
    prefix each file holds, and one background writer so saving never stalls the decode loop."""

    def __init__(self):
        self._loaded: Dict[str, float] = {}
        self._saved: Dict[str, tuple] = {}   # path -> token prefix it holds (or is being written)
        self._pending: Dict[str, tuple] = {}  # path -> newest snapshot not yet written
        self._mu = threading.Lock()
        self._cv = threading.Condition(self._mu)
        self._writer = None
        self._scratch = -(1 << 40)

    def ensure_loaded(self, engine, path: str) -> int:
        self.flush(path)
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
        """Queue a save of `tokens`' whole KV blocks.  Skipped when the file already holds that
        exact prefix; when several requests finish before the writer runs, the newest wins
        (one file per model config, as with llama.cpp session files)."""
        bs = engine.kv.block_size
        key = tuple(tokens[:len(tokens) // bs * bs])
        if not key:
            return 0
        with self._mu:
            if self._saved.get(path) == key:
                return 0
        snap = snapshot(engine, sid, tokens)
        if snap is None:
            return 0
        with self._cv:
            self._saved[path] = key
            self._pending[path] = (_meta(engine), snap)
            if self._writer is None or not self._writer.is_alive():
                self._writer = threading.Thread(target=self._write_loop, name="prompt-cache-writer", daemon=True)
                self._writer.start()
            self._cv.notify_all()
        return len(key)

    def _write_loop(self):
        while True:
            with self._cv:
                while not self._pending:
                    if not self._cv.wait(timeout=30):
                        self._writer = None
                        return
                path, (meta, snap) = next(iter(self._pending.items()))
            try:
                write(meta, snap, path)
                mt = os.path.getmtime(path)
            except Exception:
                log.exception("saving prompt cache %s", path)
                mt = None
            with self._cv:
                if self._pending.get(path, (None, None))[1] is snap:
                    del self._pending[path]
                if mt is not None:
                    self._loaded[path] = mt  # our own KV is already resident
                self._cv.notify_all()

    def flush(self, path: str = None, timeout: float = 60.0) -> None:
        """Wait until `path` (or every path) has no queued write."""
        with self._cv:
            self._cv.wait_for(lambda: not (path in self._pending if path else self._pending), timeout=timeout)
