"""LoRA adapters (model-config `lora_adapter` / `lora_base` / `lora_scale`).

Reference semantics: the llama backend takes `LoraAdapter` relative to the model's directory,
only when `LoraBase` is also set, with scale `LoraScale` (1.0 when 0)
(`backend/cpp/llama/grpc-server.cpp:2263-2271`), and hands it to llama.cpp, which reads
llama.cpp's GGUF adapter format: `general.type = "adapter"`, `adapter.type = "lora"`,
`adapter.lora.alpha`, and per adapted weight the pair `<weight name>.lora_a` [r, K] and
`<weight name>.lora_b` [N, r]; the effective delta is `scale * alpha / r * B @ A`
(`scale` alone when alpha is 0) [external: llama.cpp @ d5cb868 src/llama.cpp
llama_lora_adapter_init / llm_build_lora_mm].

Here the delta is merged at load time: an adapted weight is dequantised, the deltas of every
adapter are added in fp32, and the result is kept as a BF16 weight (the skinny / mid / library
GEMM paths all take BF16), so the forward pass runs unchanged with no per-token adapter GEMMs.
llama.cpp instead adds B(Ax) next to the quantised base GEMM at run time; the two differ by the
bf16 rounding of the merged weight.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

from ..gguf import GGUFReader, dequantize


class LoraSet:
    """Deltas of one or more LoRA adapters, keyed by the base tensor name."""

    def __init__(self, adapters: Sequence[Tuple[str, float]]):
        self.deltas: Dict[str, List[Tuple[np.ndarray, np.ndarray, float]]] = {}
        self.paths: List[str] = []
        for path, user_scale in adapters:
            self._load(path, float(user_scale) if user_scale else 1.0)

    def _load(self, path: str, user_scale: float):
        r = GGUFReader(path)
        gtype = str(r.kv.get("general.type", "adapter"))
        atype = str(r.kv.get("adapter.type", "lora"))
        if gtype != "adapter" or atype != "lora":
            raise ValueError(f"{path}: not a LoRA adapter GGUF (general.type={gtype}, adapter.type={atype})")
        alpha = float(r.kv.get("adapter.lora.alpha", 0.0) or 0.0)
        found = 0
        for name, t in r.tensors.items():
            if not name.endswith(".lora_a"):
                continue
            base = name[: -len(".lora_a")]
            tb = r.tensors.get(base + ".lora_b")
            if tb is None:
                raise ValueError(f"{path}: {name} has no matching .lora_b")
            a = dequantize(t.data, t.ggml_type, t.shape).reshape(t.shape).astype(np.float32)    # [r, K]
            b = dequantize(tb.data, tb.ggml_type, tb.shape).reshape(tb.shape).astype(np.float32)  # [N, r]
            rank = a.shape[0]
            if b.shape[1] != rank:
                raise ValueError(f"{path}: {base} lora_a rank {rank} != lora_b rank {b.shape[1]}")
            scale = user_scale * alpha / rank if alpha else user_scale
            self.deltas.setdefault(base, []).append((a, b, scale))
            found += 1
        if not found:
            raise ValueError(f"{path}: adapter holds no lora_a / lora_b tensor pairs")
        self.paths.append(path)

    def __contains__(self, name: str) -> bool:
        return name in self.deltas

    def __len__(self) -> int:
        return len(self.deltas)

    def merged(self, name: str, w: np.ndarray) -> np.ndarray:
        """w [N, K] fp32 + every adapter's delta for `name`."""
        out = np.array(w, dtype=np.float32, copy=True)
        for a, b, scale in self.deltas[name]:
            if b.shape[0] != out.shape[0] or a.shape[1] != out.shape[1]:
                raise ValueError(f"LoRA delta for {name} is {b.shape[0]}x{a.shape[1]}, weight is {out.shape}")
            out += scale * (b @ a)
        return out


def adapter_path(model_path: str, adapter: str) -> str:
    """The reference resolves the adapter against the model file's directory."""
    if os.path.isabs(adapter):
        return adapter
    return os.path.join(os.path.dirname(os.path.abspath(model_path)), adapter)
