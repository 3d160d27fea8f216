"""GPU-resident vector store (the reference's `local-store` backend, `backend/go/stores/store.go`).

The reference keeps keys as sorted Go slices and scans them on the CPU with a priority queue
(store.go:369-470).  Here the keys live as one contiguous fp32 matrix in HBM; StoresFind is a
single GEMV (`keys @ q`) + `topk` on the device, so a million 1k-dim keys is a ~4 GB matrix and a
~1 ms query on MI355X.  Exact-key lookups (Set/Get/Delete) go through a host hash map of the key
bytes -> row, with swap-remove compaction.

Semantics kept from the reference: all keys share one length (first Set fixes it), Set replaces
values of existing keys, Find returns the TopK most similar (cosine; dot product when both sides
are unit-norm), TopK >= 1, Get omits keys that are not present.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch


class VectorStore:
    def __init__(self, device: Optional[str] = None, capacity: int = 1024):
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self._lock = threading.Lock()
        self.key_len = -1
        self._keys: Optional[torch.Tensor] = None   # [cap, D] fp32
        self._norms: Optional[torch.Tensor] = None  # [cap]
        self._cap = capacity
        self._n = 0
        self._row: Dict[bytes, int] = {}
        self._vals: List[bytes] = []
        self._host_keys: List[np.ndarray] = []

    def __len__(self) -> int:
        return self._n

    @staticmethod
    def _kb(k: np.ndarray) -> bytes:
        return k.astype(np.float32).tobytes()

    def _check(self, keys: Sequence[Sequence[float]], what: str):
        if not keys:
            raise ValueError(f"no keys to {what}")
        ln = len(keys[0])
        for k in keys:
            if len(k) != ln:
                raise ValueError("all keys must have the same length")
        if self.key_len >= 0 and ln != self.key_len:
            raise ValueError(f"Try to {what} key with length {ln} when existing length is {self.key_len}")
        return ln

    def _grow(self, need: int):
        if self._keys is not None and need <= self._keys.shape[0]:
            return
        cap = max(self._cap, 1)
        while cap < need:
            cap *= 2
        nk = torch.zeros(cap, self.key_len, dtype=torch.float32, device=self.device)
        nn = torch.zeros(cap, dtype=torch.float32, device=self.device)
        if self._keys is not None and self._n:
            nk[:self._n] = self._keys[:self._n]
            nn[:self._n] = self._norms[:self._n]
        self._keys, self._norms, self._cap = nk, nn, cap

    def set(self, keys: Sequence[Sequence[float]], values: Sequence[bytes]):
        if len(keys) != len(values):
            raise ValueError(f"len(keys) = {len(keys)}, len(values) = {len(values)}")
        with self._lock:
            ln = self._check(keys, "add")
            if self.key_len < 0:
                self.key_len = ln
            new_rows, new_keys = [], []
            for k, v in zip(keys, values):
                a = np.asarray(k, dtype=np.float32)
                kb = self._kb(a)
                r = self._row.get(kb)
                if r is not None:
                    self._vals[r] = bytes(v)
                    continue
                r = self._n + len(new_rows)
                self._row[kb] = r
                self._vals.append(bytes(v))
                self._host_keys.append(a)
                new_rows.append(r)
                new_keys.append(a)
            if new_keys:
                self._grow(self._n + len(new_keys))
                t = torch.from_numpy(np.stack(new_keys)).to(self.device)
                self._keys[self._n:self._n + len(new_keys)] = t
                self._norms[self._n:self._n + len(new_keys)] = t.norm(dim=1)
                self._n += len(new_keys)

    def delete(self, keys: Sequence[Sequence[float]]):
        with self._lock:
            self._check(keys, "delete")
            for k in keys:
                r = self._row.pop(self._kb(np.asarray(k, dtype=np.float32)), None)
                if r is None:
                    continue
                last = self._n - 1
                if r != last:  # swap-remove
                    self._keys[r] = self._keys[last]
                    self._norms[r] = self._norms[last]
                    self._vals[r] = self._vals[last]
                    self._host_keys[r] = self._host_keys[last]
                    self._row[self._kb(self._host_keys[r])] = r
                self._vals.pop()
                self._host_keys.pop()
                self._n -= 1

    def get(self, keys: Sequence[Sequence[float]]) -> Tuple[List[List[float]], List[bytes]]:
        with self._lock:
            if not keys or self._n == 0:
                return [], []
            self._check(keys, "get")
            ok, ov = [], []
            for k in keys:
                a = np.asarray(k, dtype=np.float32)
                r = self._row.get(self._kb(a))
                if r is not None:
                    ok.append(a.tolist())
                    ov.append(self._vals[r])
            return ok, ov

    def find(self, key: Sequence[float], top_k: int) -> Tuple[List[List[float]], List[bytes], List[float]]:
        if top_k < 1:
            raise ValueError(f"opts.TopK = {top_k}, must be >= 1")
        with self._lock:
            if self._n == 0:
                return [], [], []
            if len(key) != self.key_len:
                raise ValueError(f"Try to find key with length {len(key)} when existing length is {self.key_len}")
            q = torch.tensor(key, dtype=torch.float32, device=self.device)
            qn = q.norm().clamp_min(1e-30)
            sims = (self._keys[:self._n] @ q) / (self._norms[:self._n].clamp_min(1e-30) * qn)
            k = min(top_k, self._n)
            s, idx = torch.topk(sims, k)
            s, idx = s.tolist(), idx.tolist()
            return [self._host_keys[i].tolist() for i in idx], [self._vals[i] for i in idx], s
