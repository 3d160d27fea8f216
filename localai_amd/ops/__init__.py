"""Operator layer: HIP (gfx950) kernels via a C ABI, plus fp32 PyTorch references.

Dispatch rule: a tensor on a GPU runs the hand-written HIP kernel from
`_la_kernels.so` -- there is NO silent eager fallback on the GPU (a missing library
raises).  CPU tensors run the PyTorch reference, which is also the numerics oracle
for the GPU tests (tests/test_kernels_gpu.py).

Every wrapper validates shapes/dtypes/contiguity on the host before launching, so a
bad call fails in Python instead of faulting the device.
"""
from __future__ import annotations

import ctypes
import functools
import math
import os
import threading
import warnings
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..gguf import GGMLType, dequantize

_LIB = None
_LIB_LOCK = threading.Lock()

FMT_Q8_0, FMT_Q4_K, FMT_Q6_K, FMT_BF16 = 8, 12, 14, 30


def lib():
    """Load (building if needed) the kernel library.  Raises if unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LIB_LOCK:
        if _LIB is not None:
            return _LIB
        from . import _build
        path = _build.LIB
        alt = os.environ.get("LOCALAI_AMD_KLIB")  # an A/B build of the same sources (_build.build_variant)
        if alt:
            path = _build.HERE / alt
        elif not path.exists() or os.environ.get("LOCALAI_AMD_REBUILD"):
            _build.build()
        L = ctypes.CDLL(str(path))
        P, I, F, LNG = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
        sig = {
            "la_qgemm_skinny": [I, P, P, P, P, I, I, P, I, I, I, P, I, LNG, P],
            "la_qgemv_dp4": [I, P, P, P, I, P, I, I, I, P, I, LNG, P, LNG, I, P, I, P],
            "la_moe_gemv": [I, I, P, I, I, I, P, I, I, P, I, I, P, LNG, I, I, P, P, I, LNG, P],
            "la_gemv_variant": [I],
            "la_moe_tune": [I, I],
            "la_dec_one_part": [I],
            "la_gather_rows": [P, P, LNG, P, P, LNG, P],
            "la_qgemv_dp4_rope": [I, P, P, P, I, P, I, P, P, P, I, I, I, P, P, P, I, P],
            "la_qgemv_dp4_norm": [I, P, P, P, I, I, I, P, I, LNG, P, P, LNG, I, P, P, F, P, P],
            "la_qgemv_dp4_rope_norm": [I, P, P, P, I, I, P, P, P, I, I, I, P, P, P, I, P, P, LNG, I, P, P, F,
                                       P, P],
            "la_add_norm": [P, P, LNG, I, P, I, P, P, P, I, I, F, I, P, P],
            "la_add_norm_router": [P, P, LNG, I, P, I, P, P, P, I, I, F, I, P, I, I, I, F, I, I, P, P, P],
            "la_rope_kv": [P, LNG, I, P, P, P, P, I, I, I, I, I, I, P, P, P, I, P],
            "la_mamba_conv_step": [P, P, LNG, P, P, P, I, I, I, P],
            "la_groupnorm_nhwc": [P, P, P, P, P, I, I, I, I, I, I, F, I, P],
            "la_mamba_ssm_step": [P, P, P, P, LNG, I, I, P, P, P, LNG, P, I, I, I, P],
            "la_act": [P, LNG, I, P, P, I, I, I, P],
            "la_reduce_slabs": [P, LNG, I, P, I, I, P, P, P],
            "la_embed": [I, P, P, P, P, I, I, P, I, P, F, P],
            "la_dequant": [I, P, P, P, P, I, I, P, P],
            "la_attn_decode": [P, P, P, P, I, P, I, I, I, I, I, F, I, I, P, P, P, P, P, LNG, I, P, P, P, P, F, I, I, P],
            "la_attn_prefill": [P, P, P, P, I, P, P, P, I, I, I, I, I, F, P, F, I, P],
            "la_sample": [P, LNG, I, I, P, P, P, P, P],
            "la_penalties": [P, LNG, I, P, I, P, P, I, P, P],
            "la_penalties_cols": [P, LNG, I, P, I, P, P, I, P, I, I, P],
            "la_tp_topc": [P, LNG, I, I, I, I, P, P],
            "la_tp_mirostat": [I, P, LNG, I, I, I, I, I, P, P, P, P, P, P, P, P],
            "la_grammar_mask": [P, LNG, I, I, P, P, LNG, P],
            "la_grammar_advance": [P, P, P, I, I, P],
            "la_sample_row_bytes": [],
            "la_logit_bias": [P, LNG, P, P, P, P, I, P],
            "la_moe_route": [P, I, I, I, P, P, P],
            "la_moe_router": [P, I, P, I, I, I, I, I, F, I, I, P, P, P],
            "la_moe_gemm": [I, I, P, I, I, I, P, P, I, P, I, I, I, P, P, I, LNG, I, P],
            "la_qw_size": [],
            "la_gemm_scales": [I, P, P, I, I, P, P],
            "la_qgemm_tile": [I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, I, P],
            "la_qgemm_tile_probe": [P, P, I, I, P, I, I, P, I, I, P],
            "la_qgemm_tile2": [I, P, P, P, I, I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, P],
            "la_pen_push": [P, I, P, I, P, P, P, P],
            "la_qgemm_glu": [I, P, P, P, I, P, P, P, I, I, I, P, I, I, P, I, I, I, P],
            "la_qgemm32": [I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, P],
            "la_moe32": [I, I, P, I, I, I, P, P, I, P, I, I, I, P, P, I, LNG, I, I, P],
            "la_moe32_probe": [I, P, I, I, I, P, P, I, P, I, I, P, I, P],
            "la_qgemm32_2": [I, P, P, P, I, I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, P],
            "la_qgemm32_glu": [I, P, P, P, I, P, P, P, I, I, I, P, I, I, P, I, I, I, P],
            "la_qgemm32_probe": [I, I, P, P, I, I, P, I, I, P, P],
            "la_attn_dense": [P, LNG, P, LNG, P, LNG, P, LNG, P, I, P, I, I, I, F, P],
            "la_bsgemm": [I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, P],
            "la_bsgemm2": [I, P, P, P, I, I, P, P, P, I, I, P, I, I, I, P, I, LNG, I, I, P],
            "la_bsgemm_glu": [I, P, P, P, I, P, P, P, I, I, I, P, I, I, P, I, I, I, P],
            "la_bsmoe": [I, I, P, I, I, I, P, P, I, P, I, I, I, P, P, I, LNG, I, I, P],
            "la_decode_advance": [P, P, P, P, P, P, I, I, I, P, I, P, P, P],
            "la_img_resample_h": [P, I, I, P, I, P, P, I, P],
            "la_img_resample_v_tiles": [P, I, I, P, P, I, I, I, I, I, I, I, P, P, P, P, P],
        }
        missing = []
        for name, args in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                # a library older than these bindings (an A/B build, a stale .so): everything else
                # still binds; calling the missing entry point fails loudly (ctypes AttributeError)
                missing.append(name)
                continue
            fn.argtypes = args
            fn.restype = I
        if missing:
            import warnings
            warnings.warn(f"{path.name} lacks {', '.join(missing)}: rebuild it (python -c 'from localai_amd.ops "
                          f"import _build; _build.build()')")
        L.la_gemm_scales_bytes.argtypes = [I, I]
        L.la_gemm_scales_bytes.restype = LNG
        gv = os.environ.get("LOCALAI_AMD_GEMV_VARIANT")
        if gv is not None:
            _check(L.la_gemv_variant(int(gv)), "la_gemv_variant")
        mt = os.environ.get("LOCALAI_AMD_MOE_TUNE")  # "row_tile,waves" of the wide-batch MoE GEMM (A/B)
        if mt:
            a, b = (int(v) for v in mt.split(","))
            _check(L.la_moe_tune(a, b), "la_moe_tune")
        if os.environ.get("LOCALAI_AMD_DEC_ONE_PART") and hasattr(L, "la_dec_one_part"):
            _check(L.la_dec_one_part(int(os.environ["LOCALAI_AMD_DEC_ONE_PART"])), "la_dec_one_part")
        _LIB = L
        return L


def hip_available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


# ---------------------------------------------------------------------------------------
# Quantised weights
# ---------------------------------------------------------------------------------------

@dataclass
class QWeight:
    """A [N, K] matrix in a runtime layout (see csrc/qweight.h)."""
    fmt: int
    N: int
    K: int
    planes: Tuple[Optional[torch.Tensor], ...]   # p0..p3 device planes (GPU path)
    ref: Optional[torch.Tensor] = None            # fp32 [N, K] (CPU path / oracle)
    bf16: Optional[torch.Tensor] = None           # optional HBM-resident bf16 copy (prefill GEMMs)
    gsc: Optional[torch.Tensor] = None            # blocked per-(column, K-step) scale plane (gemm_q.hip)

    @property
    def device(self) -> torch.device:
        t = self.planes[0] if self.planes and self.planes[0] is not None else self.ref
        return t.device

    @property
    def nbytes(self) -> int:
        return sum(p.numel() * p.element_size() for p in self.planes if p is not None)

    @staticmethod
    def from_raw(raw: np.ndarray, ggml_type: int, shape: Tuple[int, int], device: torch.device,
                 keep_ref: bool = False) -> "QWeight":
        """raw: uint8 GGUF payload of a [N, K] tensor."""
        N, K = int(shape[0]), int(shape[1])
        t = int(ggml_type)
        if device.type != "cuda":
            ref = torch.from_numpy(dequantize(raw, t, (N, K)).astype(np.float32))
            fmt = {GGMLType.Q4_K: FMT_Q4_K, GGMLType.Q6_K: FMT_Q6_K, GGMLType.Q8_0: FMT_Q8_0}.get(t, FMT_BF16)
            return QWeight(fmt, N, K, (None, None, None, None), ref=ref)
        ref = torch.from_numpy(dequantize(raw, t, (N, K)).astype(np.float32)) if keep_ref else None
        with warnings.catch_warnings():
            # raw is usually a read-only view of the mmapped GGUF; the host tensor is only read
            # by the device copy, so wrap it without a host-side copy of the payload
            warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
            src = torch.from_numpy(np.ascontiguousarray(raw)).to(device, non_blocking=False)
        if t == GGMLType.Q4_K and K % 256 == 0:
            b = src.view(N, K // 256, 144)
            qs = b[:, :, 16:].contiguous().view(N, K // 2)
            hdr = b[:, :, :16].contiguous().view(N, K // 256 * 16)
            scm, dd = _q4k_gemv_planes(b[:, :, :16])
            return QWeight(FMT_Q4_K, N, K, (qs, hdr, scm, dd), ref=ref)
        if t == GGMLType.Q6_K and K % 256 == 0:
            b = src.view(N, K // 256, 210)
            ql = b[:, :, :128].contiguous().view(N, K // 2)
            qh = b[:, :, 128:192].contiguous().view(N, K // 4)
            sc = b[:, :, 192:208].contiguous().view(N, K // 16)
            d = b[:, :, 208:210].contiguous().view(N, K // 256 * 2)
            return QWeight(FMT_Q6_K, N, K, (ql, qh, sc, d), ref=ref)
        if t == GGMLType.Q8_0 and K % 256 == 0:
            b = src.view(N, K // 32, 34)
            d = b[:, :, :2].contiguous().view(N, K // 32 * 2)
            qs = b[:, :, 2:].contiguous().view(N, K)
            return QWeight(FMT_Q8_0, N, K, (qs, d, None, None), ref=ref)
        # anything else: materialise bf16 (dequantised on the host once)
        w = torch.from_numpy(dequantize(raw, t, (N, K)).astype(np.float32)).to(device).to(torch.bfloat16)
        return QWeight(FMT_BF16, N, K, (w.view(torch.uint8).view(N, K * 2), None, None, None), ref=ref)

    @staticmethod
    def from_float(w: torch.Tensor) -> "QWeight":
        """Dense bf16 weight (used for tensors stored as F16/F32 or built in memory)."""
        N, K = w.shape
        if w.device.type != "cuda":
            return QWeight(FMT_BF16, N, K, (None, None, None, None), ref=w.float())
        wb = w.to(torch.bfloat16).contiguous()
        return QWeight(FMT_BF16, N, K, (wb.view(torch.uint8).view(N, K * 2), None, None, None))

    def ptrs(self):
        return [_ptr(p) for p in self.planes]

    @property
    def gemv_ok(self) -> bool:
        """Has the planes the int8-dot decode GEMV (gemv_dp4.hip) reads."""
        return (self.fmt == FMT_Q6_K or (self.fmt == FMT_Q4_K and self.planes[2] is not None)
                or (self.fmt == FMT_Q8_0 and self.planes[1] is not None)) and self.K % 256 == 0

    def materialize_bf16(self) -> torch.Tensor:
        """HBM-resident bf16 copy for the large-M (prefill) GEMM path."""
        if self.bf16 is None:
            if self.device.type != "cuda":
                self.bf16 = self.ref.to(torch.bfloat16)
            elif self.fmt == FMT_BF16:
                self.bf16 = self.planes[0].view(torch.bfloat16).view(self.N, self.K)
            else:
                out = torch.empty(self.N, self.K, dtype=torch.bfloat16, device=self.device)
                _check(lib().la_dequant(self.fmt, *self.ptrs(), self.N, self.K, out.data_ptr(), _stream()),
                       "la_dequant")
                self.bf16 = out
        return self.bf16

    @property
    def tile_ok(self) -> bool:
        """Can feed the quantised tile GEMM (gemm_q.hip)."""
        return self.K % 256 == 0 and self.fmt in (FMT_Q4_K, FMT_Q6_K, FMT_Q8_0, FMT_BF16) and self.planes[0] is not None

    def tile_planes(self) -> Tuple[int, Optional[int], Optional[int]]:
        """(p0, p1, gsc) pointers for la_qgemm_tile; the 8-byte-per-(column, K-step) scale plane
        is built on the device on first use (0.125 B per weight)."""
        if self.fmt == FMT_BF16:
            return _ptr(self.planes[0]), None, None
        if self.gsc is None:
            nbytes = int(lib().la_gemm_scales_bytes(self.N, self.K))
            g = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            if self.fmt == FMT_Q4_K:
                if self.planes[2] is None:
                    raise ValueError("Q4_K weight without its unpacked scale planes")
                a, b = self.planes[2], self.planes[3]
            elif self.fmt == FMT_Q6_K:
                a, b = self.planes[2], self.planes[3]
            else:
                a, b = self.planes[1], None
            _check(lib().la_gemm_scales(self.fmt, _ptr(a), _ptr(b), self.N, self.K, g.data_ptr(), _stream()),
                   "la_gemm_scales")
            self.gsc = g
        p1 = _ptr(self.planes[1]) if self.fmt == FMT_Q6_K else None
        return _ptr(self.planes[0]), p1, self.gsc.data_ptr()

    def dequant_f32(self) -> torch.Tensor:
        if self.ref is not None:
            return self.ref
        return self.materialize_bf16().float()

    def shard(self, dim: int, rank: int, world: int) -> "QWeight":
        """Row (dim=0) or column (dim=1) shard for tensor parallelism.  Column shards
        must stay aligned to 256-wide super-blocks."""
        if world == 1:
            return self
        if dim == 0:
            n = self.N // world
            sl = slice(rank * n, (rank + 1) * n)
            planes = tuple(None if p is None else p[sl].contiguous() for p in self.planes)
            ref = None if self.ref is None else self.ref[sl].contiguous()
            return QWeight(self.fmt, n, self.K, planes, ref=ref)
        k = self.K // world
        if k % 256:
            raise ValueError(f"column shard {k} not a multiple of 256")
        ref = None if self.ref is None else self.ref[:, rank * k:(rank + 1) * k].contiguous()
        planes = []
        for p in self.planes:
            if p is None:
                planes.append(None)
                continue
            per_row = p.shape[1]
            c = per_row // world
            planes.append(p[:, rank * c:(rank + 1) * c].contiguous())
        return QWeight(self.fmt, self.N, k, tuple(planes), ref=ref)


def _q4k_gemv_planes(h: torch.Tensor):
    """From Q4_K block headers h [N, nsb, 16] (f16 d, f16 dmin, 12 packed 6-bit scales/mins)
    build the two planes the decode GEMV reads: scm [N, nsb*16] = (sc0,m0,sc1,m1,...) and
    dd [N, nsb*4] = (d, dmin).  Unpacking is ggml's get_scale_min_k4 [external, llama.cpp
    ggml-quants.c], done once at load instead of per lane per step."""
    N, nsb, _ = h.shape
    q = h[:, :, 4:16].to(torch.int32)
    sc = torch.empty(N, nsb, 8, dtype=torch.int32, device=h.device)
    mn = torch.empty_like(sc)
    sc[..., :4] = q[..., 0:4] & 63
    mn[..., :4] = q[..., 4:8] & 63
    sc[..., 4:] = (q[..., 8:12] & 0xF) | ((q[..., 0:4] >> 6) << 4)
    mn[..., 4:] = (q[..., 8:12] >> 4) | ((q[..., 4:8] >> 6) << 4)
    scm = torch.stack([sc, mn], -1).to(torch.uint8).reshape(N, nsb * 16).contiguous()
    dd = h[:, :, :4].contiguous().view(N, nsb * 4)
    return scm, dd


def concat_rows(ws: Sequence[QWeight]) -> Optional[QWeight]:
    """Fuse weights with equal format and K along N (QKV, gate|up).  None if impossible."""
    if not ws or len({(w.fmt, w.K) for w in ws}) != 1:
        return None
    w0 = ws[0]
    planes = []
    for i in range(4):
        ps = [w.planes[i] for w in ws]
        planes.append(None if ps[0] is None else torch.cat(ps, 0))
    ref = None if w0.ref is None else torch.cat([w.ref for w in ws], 0)
    return QWeight(w0.fmt, sum(w.N for w in ws), w0.K, tuple(planes), ref=ref)


def fuse_runs(ws: Sequence[QWeight]) -> List[QWeight]:
    """Concatenate each run of consecutive weights that share format and K (one GEMM launch
    per run); the output column order is unchanged."""
    out: List[QWeight] = []
    run: List[QWeight] = []
    for w in ws:
        if run and (w.fmt, w.K) != (run[0].fmt, run[0].K):
            out.append(concat_rows(run) if len(run) > 1 else run[0])
            run = []
        run.append(w)
    if run:
        out.append(concat_rows(run) if len(run) > 1 else run[0])
    return out


# ---------------------------------------------------------------------------------------
# Partial results: S fp32 split-K slabs [S, M, N] or one bf16/fp32 [M, N] matrix
# ---------------------------------------------------------------------------------------

@dataclass
class Partial:
    t: torch.Tensor              # [S, M, N] f32 or [M, N] bf16/f32
    bias: Optional[torch.Tensor] = None

    @property
    def S(self) -> int:
        return self.t.shape[0] if self.t.dim() == 3 else 0

    @property
    def M(self) -> int:
        return self.t.shape[-2]

    @property
    def N(self) -> int:
        return self.t.shape[-1]

    def src_args(self):
        if self.t.dim() == 3:
            assert self.t.dtype == torch.float32
            return (self.t.data_ptr(), self.t.shape[1] * self.t.shape[2], self.t.shape[0], _ptr(self.bias))
        assert self.t.dtype == torch.bfloat16, "single-matrix sources must be bf16"
        return (self.t.data_ptr(), 0, 0, _ptr(self.bias))

    def dense(self) -> torch.Tensor:
        x = self.t.float().sum(0) if self.t.dim() == 3 else self.t.float()
        if self.bias is not None:
            x = x + self.bias.float()
        return x

    def cols(self, a: int, b: int) -> "Partial":
        t = self.t[..., a:b].contiguous()
        bias = None if self.bias is None else self.bias[a:b]
        return Partial(t, bias)


def pick_splits(N: int, K: int, M: int) -> int:
    """Split-K so the skinny GEMM launches >= ~2 workgroups per CU (256 CUs)."""
    nsb = K // 256
    nblk = (N + 63) // 64
    want = max(1, math.ceil(512 / nblk))
    best = 1
    for s in range(1, nsb + 1):
        if nsb % s == 0:
            best = s
            if s >= want:
                break
    # the consumer reads S slabs: keep the slab traffic below the weight traffic
    while best > 1 and best * M * N * 4 * 2 > N * K // 2:
        cands = [s for s in range(1, best) if nsb % s == 0]
        best = cands[-1] if cands else 1
    return best


GEMV_MAX_SPLITS = int(os.environ.get("LOCALAI_AMD_GEMV_MAX_SPLITS", "0"))   # 0: no cap (A/B knob)


def _gemv_splits(ws, K: int, M: int) -> int:
    """Split-K for the dp4 GEMV: ~2 workgroups per CU (pick_splits), then grown until the
    workgroup's int8 activation image (kper bytes + 16-run sums + scales per row) fits 64 KiB."""
    nsb = K // 256
    S = min(pick_splits(w.N, w.K, M) for w in ws)
    if all(w.fmt == FMT_Q8_0 for w in ws):
        # 1.06 B/weight (vs 0.56 for Q4_K): each split already streams twice the bytes, and half
        # the splits measured fastest (Llama-3-8B Q8_0, M=1: o 9.7 -> 7.8 us, q|k|v 12.7 -> 9.8 us)
        S = max(1, S // 2)
    if M == 1 and K >= 24576:
        # 70B-class down projections (K = 28672): 7 splits measured 9 % faster than 4 for Q6_K and
        # 4 % for Q4_K (profiles/r3_session2_measurements.md, scripts/gemv_sweep.py --preset 70b)
        S = max(S, 7)
    if GEMV_MAX_SPLITS:
        S = min(S, GEMV_MAX_SPLITS)
    while nsb % S:
        S -= 1
    mt = 1 if M == 1 else (2 if M == 2 else 4)
    while mt * (K // S) * (1 + 4 / 16 + 4 / 32) > 65536:
        S = next(s for s in range(S + 1, nsb + 1) if nsb % s == 0)
    return S


def gemv_dp4(x: Optional[torch.Tensor], ws: Sequence[QWeight], S: int, out: torch.Tensor,
             act_src: Optional[Partial] = None, act_mode: int = 0) -> None:
    """out[S, M, sum(N)] = split-K partials of x @ [W0; W1; ...]^T from the int8-dot decode GEMV,
    up to 3 weights (mixed Q4_K / Q6_K, same K) per launch.  With act_src (fp32 gate|up slabs)
    x = act(act_src) is formed inside the GEMV prologue instead of being read."""
    M = out.shape[1]
    K = ws[0].K
    a = (None, 0, 0, None) if act_src is None else act_src.src_args()
    Ntot = out.shape[-1]
    # launch groups: <= 3 weights whose formats form at most two runs [FA ...][FB ...]
    groups: List[List[QWeight]] = []
    for w in ws:
        g = groups[-1] if groups else None
        if (g is not None and len(g) < 3 and (len({v.fmt for v in g}) == 1 or w.fmt == g[-1].fmt)
                and (w.fmt == FMT_Q8_0) == (g[0].fmt == FMT_Q8_0)):  # Q8_0 launches are homogeneous
            g.append(w)
        else:
            groups.append([w])
    col = 0
    for seg in groups:
        n = len(seg)
        fmts = (ctypes.c_int * n)(*[w.fmt for w in seg])
        planes = (ctypes.c_void_p * (4 * n))(*[p for w in seg for p in w.ptrs()])
        Ns = (ctypes.c_int * n)(*[w.N for w in seg])
        args = (n, fmts, planes, Ns, K, None if x is None else x.data_ptr(), K, M, S, out.data_ptr() + col * 4,
                Ntot, M * Ntot, a[0], a[1], a[2], a[3], act_mode)
        _check(lib().la_qgemv_dp4(*args, _stream()), "la_qgemv_dp4")
        col += sum(w.N for w in seg)


# off by default: measured neutral on Llama-3-8B C=1 (profiles/r4_c1_fused_norm.md) -- the 33
# add_norm launches go away, but every q|k|v workgroup re-reads the residual plus the down
# projection's 8 split-K slabs (144 KiB from L2 per workgroup) and the GEMV grows by the same ~4 us
GEMV_NORM = os.environ.get("LOCALAI_AMD_GEMV_NORM", "0") == "1"


@dataclass
class NormIn:
    """A deferred layer-boundary residual-add + RMSNorm, handed to the consuming decode GEMV
    instead of a materialised bf16 x: x = rmsnorm(res + add) * weight is formed in the GEMV
    prologue (gemv_dp4.hip GV_NORM) and the updated residual lands in res_out (written once, by
    one workgroup; None when there is no add).  Removes the add_norm launch at every layer
    boundary of a batch-1/2 decode step (SURVEY §2.8 K2 + K14 folded into K5)."""
    res: torch.Tensor               # fp32 [M, D]
    add: Optional[Partial]          # fp32 split-K slabs [S, M, D] or None
    weight: torch.Tensor            # fp32 [D]
    eps: float
    res_out: Optional[torch.Tensor]  # fp32 [M, D], not res; None iff add is None

    @property
    def shape(self):
        return self.res.shape

    @property
    def is_cuda(self) -> bool:
        return self.res.is_cuda

    def args(self):
        a = self.add.src_args() if self.add is not None else (None, 0, 0, None)
        return (self.res.data_ptr(), a[0], a[1], a[2], a[3], self.weight.data_ptr(), float(self.eps),
                _ptr(self.res_out))

    def materialize(self) -> torch.Tensor:
        """The same x through add_norm (residual updated in res, then copied to res_out)."""
        xn = add_norm(self.res, self.add, self.weight, None, self.eps, 0)
        if self.res_out is not None:
            self.res_out.copy_(self.res)
        return xn


def norm_in_ok(res: torch.Tensor, add: Optional[Partial], weight: torch.Tensor, bias) -> bool:
    """A NormIn can feed the fused GEMV prologue: GPU, fp32 residual of <= GEMV_MAX_M rows and
    width <= 8192, fp32 weight, no norm bias (RMSNorm), the add as fp32 split-K slabs."""
    M, D = res.shape
    return (GEMV_NORM and GEMV_DP4 and res.is_cuda and res.dtype == torch.float32 and M <= GEMV_MAX_M
            and D <= 8192 and D % 256 == 0 and bias is None and weight.dtype == torch.float32
            and (add is None or (add.t.dim() == 3 and add.t.dtype == torch.float32 and add.S <= 16
                                 and add.N == D)))


def qkv_rope_ok(x: torch.Tensor, ws: Sequence[QWeight], bias, mode: int, rot: int, Dh: int, block_size: int) -> bool:
    """The fused decode q|k|v GEMV + RoPE + KV append (gemv_dp4.hip GVRope) applies: GPU, batch
    <= GEMV_MAX_M, Q4_K/Q6_K weights, no bias, NORM rotary over the whole head."""
    return (x.is_cuda and GEMV_DP4 and x.shape[0] <= GEMV_MAX_M and bias is None and mode == 0 and rot == Dh
            and Dh % 2 == 0 and block_size % 8 == 0 and len(ws) <= 3 and all(w.gemv_ok for w in ws)
            and len({w.K for w in ws}) == 1 and ws[0].K % 1024 == 0
            and len({w.fmt == FMT_Q8_0 for w in ws}) == 1)


def qkv_rope_dp4(x: torch.Tensor, ws: Sequence[QWeight], pos: torch.Tensor, slots: torch.Tensor,
                 cos_sin: torch.Tensor, Hq: int, Hkv: int, Dh: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
                 block_size: int, q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q = rope(x @ Wq^T) [M, Hq, Dh] bf16; k = rope(x @ Wk^T) and v = x @ Wv^T appended to the paged
    cache at `slots` -- one GEMV launch (split-K 1) with the rotation and the append in its
    epilogue, instead of a GEMV + rope_kv."""
    M, K = x.shape
    if isinstance(x, NormIn):
        if q_out is None:
            q_out = torch.empty(M, Hq, Dh, dtype=torch.bfloat16, device=x.res.device)
        if sum(w.N for w in ws) != (Hq + 2 * Hkv) * Dh:
            raise ValueError("qkv_rope_dp4: weights do not form q|k|v")
        n = len(ws)
        fmts = (ctypes.c_int * n)(*[w.fmt for w in ws])
        planes = (ctypes.c_void_p * (4 * n))(*[p for w in ws for p in w.ptrs()])
        Ns = (ctypes.c_int * n)(*[w.N for w in ws])
        _check(lib().la_qgemv_dp4_rope_norm(n, fmts, planes, Ns, K, M, pos.data_ptr(), slots.data_ptr(),
                                            cos_sin.data_ptr(), Hq, Hkv, Dh, q_out.data_ptr(), k_cache.data_ptr(),
                                            v_cache.data_ptr(), block_size, *x.args(), _stream()),
               "la_qgemv_dp4_rope_norm")
        return q_out
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("qkv_rope_dp4: x must be contiguous bf16")
    if sum(w.N for w in ws) != (Hq + 2 * Hkv) * Dh:
        raise ValueError("qkv_rope_dp4: weights do not form q|k|v")
    if pos.dtype != torch.int32 or slots.dtype != torch.int32 or pos.numel() < M or slots.numel() < M:
        raise ValueError("qkv_rope_dp4: pos / slots must be int32 [M]")
    if q_out is None:
        q_out = torch.empty(M, Hq, Dh, dtype=torch.bfloat16, device=x.device)
    n = len(ws)
    fmts = (ctypes.c_int * n)(*[w.fmt for w in ws])
    planes = (ctypes.c_void_p * (4 * n))(*[p for w in ws for p in w.ptrs()])
    Ns = (ctypes.c_int * n)(*[w.N for w in ws])
    _check(lib().la_qgemv_dp4_rope(n, fmts, planes, Ns, K, x.data_ptr(), M, pos.data_ptr(), slots.data_ptr(),
                                   cos_sin.data_ptr(), Hq, Hkv, Dh, q_out.data_ptr(), k_cache.data_ptr(),
                                   v_cache.data_ptr(), block_size, _stream()), "la_qgemv_dp4_rope")
    return q_out


SKINNY_MAX_M = 64
GEMV_MAX_M = 2           # M <= GEMV_MAX_M: int8-dot decode GEMV (gemv_dp4.hip, supports M <= 4) on Q4_K/Q6_K
GEMV_DP4 = os.environ.get("LOCALAI_AMD_GEMV", "dp4") == "dp4"
MID_MAX_M = 256          # 64 < M <= MID_MAX_M: quantised MFMA tile GEMMs (gemm_q.hip / gemm_q32.hip), autotuned
GEMM_AUTOTUNE = True
# (M, K, ((fmt, N), ...)) -> (kind, S, variant); filled by _autotune_mid at warm-up (eager runs
# before each decode-graph capture), consulted during capture / replay.
_GEMM_CHOICE: dict = {}


def blas_tuning_start(path: Optional[str] = None) -> bool:
    """Per-shape solution search for the library (hipBLASLt / rocBLAS) GEMMs, run while the engine
    warms up its decode graphs: PyTorch-ROCm TunableOp times every candidate kernel of each new
    (M, N, K) against a rotating 512 MiB buffer set (cold weights, as in decode) and keeps the
    fastest.  Results persist in a CSV so a restart reuses them.  Tuning is switched off again
    before serving (blas_tuning_stop): prefill chunk sizes vary and must never tune inline."""
    if os.environ.get("LOCALAI_AMD_BLAS_TUNE", "1") == "0" or not torch.cuda.is_available():
        return False
    try:
        import torch.cuda.tunable as tn
    except ImportError:
        return False
    if path is None:
        root = os.environ.get("LOCALAI_AMD_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "localai_amd")
        os.makedirs(root, exist_ok=True)
        dev = torch.cuda.current_device()
        name = torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0]
        # one file per device: data-parallel ranks on one node tune (and write) concurrently
        path = os.path.join(root, f"tunableop_{name}_dev{dev}.csv")
    tn.enable(True)
    tn.set_filename(path)
    if os.path.exists(path):
        try:
            tn.read_file(path)
        except Exception:  # noqa: BLE001 - a stale/corrupt cache only costs a re-tune
            pass
    tn.set_max_tuning_duration(int(os.environ.get("LOCALAI_AMD_BLAS_TUNE_MS", "15")))
    tn.set_max_tuning_iterations(20)
    try:
        tn.set_rotating_buffer_size(512)
    except Exception:  # noqa: BLE001
        pass
    tn.tuning_enable(True)
    return True


class blas_tuning_paused:
    """Context: library GEMMs inside run on already-tuned or default solutions without tuning new
    shapes.  For GEMMs whose M changes every step (a MoE expert's routed rows during prefill): each
    new (M, N, K) would otherwise be tuned during warm-up -- hundreds of shapes, minutes of start-up."""

    def __enter__(self):
        self.prev = False
        if not torch.cuda.is_available():
            return self
        try:
            import torch.cuda.tunable as tn
            self.prev = tn.is_enabled() and tn.tuning_is_enabled()
            if self.prev:
                tn.tuning_enable(False)
        except (ImportError, RuntimeError):
            pass
        return self

    def __exit__(self, *exc):
        if self.prev:
            import torch.cuda.tunable as tn
            tn.tuning_enable(True)
        return False


def blas_tuning_stop() -> None:
    import torch.cuda.tunable as tn
    tn.tuning_enable(False)   # keep using the tuned solutions, never tune inline while serving
    try:
        tn.write_file()
    except Exception:  # noqa: BLE001
        pass


def fuse_bf16(ws: Sequence[QWeight]) -> Optional[torch.Tensor]:
    """One HBM-resident bf16 [sum(N), K] matrix behind several weights that feed one output
    (a Q4_K q|k with a Q6_K v): each weight's bf16 copy becomes a row slice of it, so the
    library path runs ONE GEMM for the fused output instead of one per format (at decode
    batch 256 the separate v GEMM cost a launch of its own: 12.5 us x 16 layers per step).
    No extra memory: the per-weight copies are the slices."""
    if len(ws) < 2 or any(w.device.type != "cuda" or w.K != ws[0].K for w in ws):
        return None
    base = getattr(ws[0], "_fused_bf16", None)
    if base is not None and base.shape[0] == sum(w.N for w in ws):
        return base
    Ntot, K = sum(w.N for w in ws), ws[0].K
    fused = torch.empty(Ntot, K, dtype=torch.bfloat16, device=ws[0].device)
    row = 0
    for w in ws:
        fused[row:row + w.N].copy_(w.materialize_bf16())
        w.bf16 = fused[row:row + w.N]
        row += w.N
    ws[0]._fused_bf16 = fused
    return fused


_SCRATCH: dict = {}
_SCRATCH_LOCK = threading.Lock()


def _scratch(device, need: int) -> torch.Tensor:
    """bf16 dequant scratch of >= need elements for the calling thread.

    One buffer per (device, thread): two engines serving from different threads on one GPU
    (in-process whisper / CLIP / a second LLM) enqueue their dequant + GEMM pairs interleaved,
    so a shared buffer would hand one engine's GEMM the other's weights.  Entries of threads that
    have exited are dropped on the next call, so an executor pool's turnover does not keep one
    large buffer per dead thread (VRAM outside the KV budget).  Inside a stream capture the buffer
    is allocated fresh from the graph's private pool instead: a replayed graph must never write
    into memory that a later (larger) scratch reallocation returned to the caching allocator."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(need, dtype=torch.bfloat16, device=device)
    key = (device, threading.get_ident())
    with _SCRATCH_LOCK:
        buf = _SCRATCH.get(key)
        if buf is None or buf.numel() < need:
            live = {t.ident for t in threading.enumerate()}
            for k in [k for k in _SCRATCH if k[1] not in live]:
                del _SCRATCH[k]
            _SCRATCH.pop(key, None)
            buf = _SCRATCH[key] = torch.empty(need, dtype=torch.bfloat16, device=device)
    return buf


def release_scratch(device=None) -> None:
    """Drop the calling thread's dequant scratch (a non-engine caller after a large GEMM)."""
    with _SCRATCH_LOCK:
        for k in [k for k in _SCRATCH if k[1] == threading.get_ident() and (device is None or k[0] == device)]:
            del _SCRATCH[k]


def _run_scratch_blas(x, ws, Ntot):
    """Large-M (prefill chunk) GEMM: dequantise the weights into a per-thread bf16 scratch
    buffer (reused by every call, sized by the largest fused weight seen), then a library GEMM
    on it -- the reference's own large-batch path (ggml convert.cu dequant + hipBLAS GemmEx,
    SURVEY K7), without a persistent bf16 copy of the model.  The dequant streams the quantised
    bytes once and writes 2 B/weight: ~6 % of a 8192-row chunk's GEMM time.  A lone bf16 weight
    is multiplied in place (no copy)."""
    K = x.shape[1]
    if len(ws) == 1 and ws[0].fmt == FMT_BF16:
        return torch.matmul(x, ws[0].planes[0].view(torch.bfloat16).view(ws[0].N, K).t())
    need = Ntot * K
    wt = _scratch(x.device, need)[:need].view(Ntot, K)
    row = 0
    for w in ws:
        if w.fmt == FMT_BF16:
            wt[row:row + w.N].copy_(w.planes[0].view(torch.bfloat16).view(w.N, w.K))
        else:
            _check(lib().la_dequant(w.fmt, *w.ptrs(), w.N, w.K, wt[row:row + w.N].data_ptr(), _stream()), "la_dequant")
        row += w.N
    return torch.matmul(x, wt.t())


def _run_blas(x, ws, Ntot):
    if TILE_GEMM and all(w.bf16 is None for w in ws) and getattr(ws[0], "_fused_bf16", None) is None:
        return _run_scratch_blas(x, ws, Ntot)
    if len(ws) == 1:
        return torch.matmul(x, ws[0].materialize_bf16().t())
    fused = getattr(ws[0], "_fused_bf16", None)
    if fused is not None and fused.shape[0] == Ntot:
        return torch.matmul(x, fused.t())
    y = torch.empty(x.shape[0], Ntot, dtype=torch.bfloat16, device=x.device)
    col = 0
    for w in ws:
        torch.matmul(x, w.materialize_bf16().t(), out=y[:, col:col + w.N])
        col += w.N
    return y


_FLUSH: dict = {}


def _cold_caches(device):
    """Evict L2 and the 256 MiB Infinity Cache by READING a 384 MiB scratch buffer (a write
    flush leaves dirty lines whose write-back then taxes the timed call), so a timed GEMM
    reads its weights from HBM as it does in the engine, where every decode step streams the
    whole model once."""
    buf = _FLUSH.get(device)
    if buf is None:
        buf = _FLUSH[device] = torch.ones(96 << 20, dtype=torch.float32, device=device)
    buf.sum()


# Quantised tile GEMM (gemm_q.hip): the M > SKINNY_MAX_M path.  Tile ids: (BM, BN).
GQ_TILES = {0: (256, 256), 1: (256, 128), 2: (128, 256), 3: (128, 128), 4: (256, 64), 5: (64, 256), 6: (256, 256),
            7: (128, 256), 8: (256, 128), 12: (128, 128), 14: (64, 256),
            # software-pipelined schedules of 0, 1, 3, 6, 7
            10: (256, 256), 11: (256, 128), 13: (128, 128), 16: (256, 256), 17: (128, 256)}
# LOCALAI_AMD_TILE_GEMM=0 restores the round-2 path (hipBLASLt on bf16 weight copies)
TILE_GEMM = os.environ.get("LOCALAI_AMD_TILE_GEMM", "1") == "1"
# M > MID_MAX_M (prefill chunks): "blas" = dequantise into a scratch buffer + library GEMM, "tile" =
# gemm_q.hip.  "blas" stays the default: the in-kernel-dequant MFMA GEMMs (gemm_bs.hip, and round
# 5's gemm_pp.hip before it) top out near 1.0 PF/s against hipBLASLt's 1.3 at M = 8192
# (profiles/r6_gemm_bs.md, r5_prefill_gemm.md)
PREFILL_GEMM = os.environ.get("LOCALAI_AMD_PREFILL_GEMM", "blas")


def _tile_split_ok(K: int, S: int) -> bool:
    ks = K // 64
    return S >= 1 and -(-ks // S) * (S - 1) < ks


_TILE2_PAIRS = {(FMT_Q4_K, FMT_Q6_K), (FMT_Q6_K, FMT_Q4_K)}
_TILE2_TILES = (7, 8, 12)


def _run_tile(x, ws, S, out, Ntot, tile):
    """out: fp32 slabs [S, M, Ntot], or a bf16 [M, Ntot] matrix (S == 1).  Two weights of a
    Q4_K/Q6_K mix (q|k + v) run as ONE launch (la_qgemm_tile2)."""
    M, K = x.shape
    bf = out.dtype == torch.bfloat16
    esz = 2 if bf else 4
    if len(ws) == 2 and (ws[0].fmt, ws[1].fmt) in _TILE2_PAIRS and tile in _TILE2_TILES:
        a0, a1, ag = ws[0].tile_planes()
        b0, b1, bg = ws[1].tile_planes()
        _check(lib().la_qgemm_tile2(ws[0].fmt, a0, a1, ag, ws[0].N, ws[1].fmt, b0, b1, bg, ws[1].N, K, x.data_ptr(), K,
                                    M, S, out.data_ptr(), Ntot, 0 if bf else M * Ntot, int(bf), tile, _stream()),
               "la_qgemm_tile2")
        return
    col = 0
    for w in ws:
        p0, p1, g = w.tile_planes()
        _check(lib().la_qgemm_tile(w.fmt, p0, p1, g, w.N, w.K, x.data_ptr(), K, M, S, out.data_ptr() + col * esz,
                                   Ntot, 0 if bf else M * Ntot, int(bf), tile, 0, _stream()), "la_qgemm_tile")
        col += w.N


# 32x32x16 quantised GEMM (gemm_q32.hip): variant id -> (BM, BN).  Variants 2 / 6 (256 x 256
# tiles) are built for Q4_K only and not for two-weight launches.
Q32_TILES = {0: (256, 128), 1: (128, 256), 2: (256, 256), 3: (128, 128), 4: (256, 128), 5: (128, 256),
             6: (256, 256), 7: (128, 128), 8: (128, 256), 9: (128, 256)}
Q32_FMTS = (FMT_Q4_K, FMT_Q6_K, FMT_Q8_0)
Q32 = os.environ.get("LOCALAI_AMD_Q32", "1") == "1"


def q32_ok(ws: Sequence[QWeight], var: int) -> bool:
    """Can the 32x32x16 kernel run these weights (one launch per weight, or one for a Q4_K/Q6_K
    pair) in this variant."""
    if not Q32 or not all(w.fmt in Q32_FMTS and w.K % 256 == 0 and w.planes[0] is not None for w in ws):
        return False
    if var in (2, 6):
        return all(w.fmt == FMT_Q4_K for w in ws) and len(ws) == 1
    return True


def _run_q32(x, ws, S, out, Ntot, var):
    """out: fp32 slabs [S, M, Ntot], or a bf16 [M, Ntot] matrix (S == 1).  A Q4_K/Q6_K pair (q|k +
    v) runs as ONE launch (la_qgemm32_2)."""
    M, K = x.shape
    bf = out.dtype == torch.bfloat16
    esz = 2 if bf else 4
    if len(ws) == 2 and (ws[0].fmt, ws[1].fmt) in _TILE2_PAIRS:
        a0, a1, ag = ws[0].tile_planes()
        b0, b1, bg = ws[1].tile_planes()
        _check(lib().la_qgemm32_2(ws[0].fmt, a0, a1, ag, ws[0].N, ws[1].fmt, b0, b1, bg, ws[1].N, K, x.data_ptr(), K,
                                  M, S, out.data_ptr(), Ntot, 0 if bf else M * Ntot, int(bf), var, _stream()),
               "la_qgemm32_2")
        return
    col = 0
    for w in ws:
        p0, p1, g = w.tile_planes()
        _check(lib().la_qgemm32(w.fmt, p0, p1, g, w.N, w.K, x.data_ptr(), K, M, S, out.data_ptr() + col * esz, Ntot,
                                0 if bf else M * Ntot, int(bf), var, _stream()), "la_qgemm32")
        col += w.N


# Shared-dequant-image GEMM (gemm_bs.hip): variant id -> (BM, BN).  Each weight column is
# dequantised once per workgroup into an LDS image all four waves read; X arrives by full-line
# loads through a private per-wave LDS transpose.  Decode batches (M 65..256) and prefill chunks.
BS_TILES = {0: (256, 128), 1: (128, 128), 2: (256, 256), 3: (256, 128)}
BS_FMTS = (FMT_Q4_K, FMT_Q6_K, FMT_Q8_0, FMT_BF16)
BS = os.environ.get("LOCALAI_AMD_BS", "1") == "1"


def bs_ok(ws: Sequence[QWeight]) -> bool:
    """Can gemm_bs.hip run these weights (one launch per weight, or one for a Q4_K/Q6_K pair)."""
    return BS and all(w.fmt in BS_FMTS and w.K % 256 == 0 and w.N % 4 == 0 and w.planes[0] is not None
                      for w in ws)


def _bs_grid(M: int, N: int, var: int) -> int:
    bm, bn = BS_TILES[var]
    return -(-M // bm) * -(-N // bn)


def _run_bs(x, ws, S, out, Ntot, var):
    """out: fp32 slabs [S, M, Ntot], or a bf16 [M, Ntot] matrix (S == 1).  A Q4_K/Q6_K pair (q|k +
    v) runs as ONE launch (la_bsgemm2)."""
    M, K = x.shape
    bf = out.dtype == torch.bfloat16
    esz = 2 if bf else 4
    slab = 0 if bf else M * Ntot
    if len(ws) == 2 and (ws[0].fmt, ws[1].fmt) in _TILE2_PAIRS:
        a0, a1, ag = ws[0].tile_planes()
        b0, b1, bg = ws[1].tile_planes()
        _check(lib().la_bsgemm2(ws[0].fmt, a0, a1, ag, ws[0].N, ws[1].fmt, b0, b1, bg, ws[1].N, K, x.data_ptr(), K,
                                M, S, out.data_ptr(), Ntot, slab, int(bf), var, _stream()), "la_bsgemm2")
        return
    col = 0
    for w in ws:
        p0, p1, g = w.tile_planes()
        _check(lib().la_bsgemm(w.fmt, p0, p1, g, w.N, w.K, x.data_ptr(), K, M, S, out.data_ptr() + col * esz, Ntot,
                               slab, int(bf), var, _stream()), "la_bsgemm")
        col += w.N


def _run_bs_glu(x, pair, F: int, mode: int, var: int, out) -> None:
    M, K = x.shape
    wa, oa, wb, ob = pair
    a0, a1, ag = wa.tile_planes()
    b0, b1, bg = wb.tile_planes()
    _check(lib().la_bsgemm_glu(wa.fmt, a0, a1, ag, oa, b0, b1, bg, ob, F, K, x.data_ptr(), K, M, out.data_ptr(), F,
                               mode, var, _stream()), "la_bsgemm_glu")


def _q32_grid(M: int, N: int, var: int) -> int:
    bm, bn = Q32_TILES[var]
    return -(-M // bm) * -(-N // bn)


def _tile_grid(M: int, N: int, tile: int) -> int:
    bm, bn = GQ_TILES[tile]
    return -(-M // bm) * -(-N // bn)


def pick_tile(M: int, Ns: Sequence[int], K: int) -> Tuple[int, int]:
    """Heuristic (tile, split-K) for shapes the autotuner has not seen (prefill chunks): the
    largest tile that still gives >= ~192 workgroups, else split K up to ~256 workgroups with
    every split >= 8 K-steps."""
    N = max(Ns)
    ks = K // 64
    for tile in ((6, 1, 3) if M > 128 else (7, 3, 5)):
        tiles = _tile_grid(M, N, tile)
        if tiles >= 192:
            return tile, 1
    tile = 1 if M > 128 else 3
    tiles = _tile_grid(M, N, tile)
    S = max(1, min(ks // 8, round(256 / tiles)))
    while S > 1 and not _tile_split_ok(K, S):
        S -= 1
    return tile, S


def _autotune_mid(x, ws, key, Ntot):
    """Time the tile GEMM's (tile, split-K) candidates with COLD weights (caches flushed before
    every timed call, as in decode where each step streams the whole model once) and remember
    the winner.  A split variant is charged for the extra fp32 bytes its consumer reads (at
    ~4 TB/s)."""
    M, K = x.shape
    N = max(w.N for w in ws)
    cands = []
    if all(w.tile_ok for w in ws):
        tiles = (6, 1, 7, 8, 12) if M > 128 else (7, 12, 14, 3)
        for t in tiles:
            g = _tile_grid(M, N, t)
            base = max(1, round(256 / g))
            # split-K <= 8: every split costs its consumer another fp32 [M, N] slab read
            for S in sorted({1, max(1, base // 2), base, base * 2}):
                if S <= min(8, K // 256) and _tile_split_ok(K, S):
                    cands.append(("tile", S, t))
        for v in ((9, 8, 4, 6, 0) if M > 128 else (9, 8, 7, 3)):
            if not q32_ok(ws, v):
                continue
            base = max(1, round(256 / _q32_grid(M, N, v)))
            for S in sorted({1, max(1, base // 2), base, base * 2}):
                if S <= min(8, K // 256) and _tile_split_ok(K, S):
                    cands.append(("q32", S, v))
    if bs_ok(ws) and (len(ws) == 1 or (len(ws) == 2 and (ws[0].fmt, ws[1].fmt) in _TILE2_PAIRS)):
        for v in ((0, 1, 3) if M > 128 else (1,)):
            base = max(1, round(256 / _bs_grid(M, N, v)))
            for S in sorted({1, max(1, base // 2), base, base * 2}):
                if S <= min(8, K // 256) and _tile_split_ok(K, S):
                    cands.append(("bs", S, v))
    if not cands or not TILE_GEMM:
        cands = [("blas", 0, 0)]
    outs = {S: torch.empty(S, M, Ntot, dtype=torch.float32, device=x.device) for _, S, _ in cands if S > 1}
    outs[1] = torch.empty(M, Ntot, dtype=torch.bfloat16, device=x.device)   # S = 1: one bf16 matrix
    best, best_t = cands[0], float("inf")
    for kind, S, t in cands:
        if kind == "blas":
            fn = lambda: _run_blas(x, ws, Ntot)  # noqa: E731
        elif kind == "tile":
            fn = lambda S=S, t=t: _run_tile(x, ws, S, outs[S], Ntot, t)  # noqa: E731
        elif kind == "bs":
            fn = lambda S=S, t=t: _run_bs(x, ws, S, outs[S], Ntot, t)  # noqa: E731
        else:
            fn = lambda S=S, t=t: _run_q32(x, ws, S, outs[S], Ntot, t)  # noqa: E731
        fn()
        ts = []
        for _ in range(3):
            _cold_caches(x.device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        tt = sorted(ts)[1]
        if kind != "blas" and S > 1:
            # fp32 slabs: written here and read back by the consumer (vs one bf16 matrix), ~4 TB/s each way
            tt += 2 * (S * M * Ntot * 4 - M * Ntot * 2) / 4e6
        if tt < best_t:
            best, best_t = (kind, S, t), tt
    _GEMM_CHOICE[key] = best
    return best


def linear(x: torch.Tensor, w: QWeight, bias: Optional[torch.Tensor] = None,
           out_slabs: Optional[torch.Tensor] = None, force: Optional[str] = None) -> Partial:
    """y = x @ W^T.  x: [M, K] bf16.  GPU: M <= 2 -> int8-dot GEMV, M <= 64 -> skinny MFMA
    kernel, larger M -> the quantised tile GEMM (gemm_q.hip); all on the quantised weights."""
    return linear_multi(x, [w], bias, out_slabs, force)


def linear_multi(x: torch.Tensor, ws: Sequence[QWeight], bias: Optional[torch.Tensor] = None,
                 out_slabs: Optional[torch.Tensor] = None, force: Optional[str] = None) -> Partial:
    """y = x @ [W0; W1; ...]^T written side by side into ONE partial (e.g. Q4_K q|k with a
    Q6_K v), so the consumer sees a single fused QKV / gate|up output."""
    M, K = x.shape
    for w in ws:
        if K != w.K:
            raise ValueError(f"linear: x has K={K}, weight has K={w.K}")
    Ntot = sum(w.N for w in ws)
    if not x.is_cuda:
        y = torch.cat([x.float() @ w.dequant_f32().t() for w in ws], -1)
        return Partial(y.to(torch.bfloat16) if force == "bf16" else y.unsqueeze(0), bias)
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("linear: x must be contiguous bf16")
    skinny_ok = all(w.K % 256 == 0 for w in ws)
    use_skinny = (M <= SKINNY_MAX_M and skinny_ok) if force is None else force == "skinny"
    tile_ok = TILE_GEMM and all(w.tile_ok for w in ws)
    S, tile, kind = 0, 0, None
    if force is not None and (force.startswith("q32:") or force.startswith("bs:")):
        kind, v, s_ = force.split(":")
        tile, S = int(v), int(s_)
    elif force is not None and force.startswith("tile"):
        # "tile" (heuristic) or "tile:<id>:<S>"
        parts = force.split(":")
        tile, S = (int(parts[1]), int(parts[2])) if len(parts) == 3 else pick_tile(M, [w.N for w in ws], K)
        kind = "tile"
    elif force is None and not use_skinny and M <= MID_MAX_M and tile_ok:
        # one tuned choice per 32-row bucket: prefill chunk / decode batch sizes vary per step
        # and must not re-run the (cache-flushing) autotune inside the serving loop
        key = ((M + 31) // 32 * 32, K, tuple((w.fmt, w.N) for w in ws))
        choice = _GEMM_CHOICE.get(key)
        if choice is None and GEMM_AUTOTUNE and not torch.cuda.is_current_stream_capturing():
            choice = _autotune_mid(x, ws, key, Ntot)
        if choice is None and tile_ok:
            t, s_ = pick_tile(M, [w.N for w in ws], K)
            choice = ("tile", s_, t)
        if choice is not None and choice[0] in ("tile", "q32", "bs"):
            kind, S, tile = choice
    elif force is None and not use_skinny and tile_ok and PREFILL_GEMM == "tile":
        tile, S = pick_tile(M, [w.N for w in ws], K)   # prefill: heuristic, never tuned inline
        kind = "tile"
    if kind in ("tile", "q32", "bs") and S == 1 and out_slabs is None:
        y = torch.empty(M, Ntot, dtype=torch.bfloat16, device=x.device)
        {"tile": _run_tile, "q32": _run_q32, "bs": _run_bs}[kind](x, ws, 1, y, Ntot, tile)
        return Partial(y, bias)
    if S:
        out = out_slabs
        if out is None or out.shape != (S, M, Ntot):
            out = torch.empty(S, M, Ntot, dtype=torch.float32, device=x.device)
        if kind == "tile":
            _run_tile(x, ws, S, out, Ntot, tile)
        elif kind == "bs":
            _run_bs(x, ws, S, out, Ntot, tile)
        else:
            _run_q32(x, ws, S, out, Ntot, tile)
        return Partial(out, bias)
    use_gemv = (force == "dp4") or (force is None and use_skinny and GEMV_DP4 and M <= GEMV_MAX_M
                                    and all(w.gemv_ok for w in ws))
    if use_gemv:
        if M > 4 or not all(w.gemv_ok for w in ws):
            raise ValueError("linear: dp4 GEMV needs M <= 4 and Q4_K/Q6_K weights")
        S = _gemv_splits(ws, K, M)
        out = out_slabs
        if out is None or out.shape != (S, M, Ntot):
            out = torch.empty(S, M, Ntot, dtype=torch.float32, device=x.device)
        gemv_dp4(x, ws, S, out)
        return Partial(out, bias)
    if use_skinny:
        S = min(pick_splits(w.N, w.K, M) for w in ws)
        nsb = K // 256
        while nsb % S:
            S -= 1
        out = out_slabs
        if out is None or out.shape != (S, M, Ntot):
            out = torch.empty(S, M, Ntot, dtype=torch.float32, device=x.device)
        col = 0
        for w in ws:
            dst = out.data_ptr() + col * 4
            _check(lib().la_qgemm_skinny(w.fmt, *w.ptrs(), w.N, w.K, x.data_ptr(), K, M, S, dst, Ntot,
                                         M * Ntot, _stream()), "la_qgemm_skinny")
            col += w.N
        return Partial(out, bias)
    return Partial(_run_blas(x, ws, Ntot), bias)


GLU_FUSE = os.environ.get("LOCALAI_AMD_GLU_FUSE", "1") == "1"
_GLU_CHOICE: Dict[tuple, Optional[int]] = {}


def _glu_pair(ws: Sequence[QWeight], F: int):
    """(gate weight, row offset, up weight, row offset) of a gate|up projection, or None."""
    if not all(w.tile_ok for w in ws):
        return None
    if len(ws) == 2 and ws[0].N == F and ws[1].N == F and ws[0].fmt == ws[1].fmt:
        return ws[0], 0, ws[1], 0
    if len(ws) == 1 and ws[0].N == 2 * F and F % 16 == 0:
        return ws[0], 0, ws[0], F
    return None


def _run_glu(x: torch.Tensor, pair, F: int, mode: int, tile: int, out: torch.Tensor) -> None:
    """tile < 100: gemm_q.hip tile id; 100 + v: gemm_q32.hip variant v; 200 + v: gemm_bs.hip variant v."""
    M, K = x.shape
    wa, oa, wb, ob = pair
    if tile >= 200:
        _run_bs_glu(x, pair, F, mode, tile - 200, out)
        return
    a0, a1, ag = wa.tile_planes()
    b0, b1, bg = wb.tile_planes()
    if tile >= 100:
        _check(lib().la_qgemm32_glu(wa.fmt, a0, a1, ag, oa, b0, b1, bg, ob, F, K, x.data_ptr(), K, M, out.data_ptr(),
                                    F, mode, tile - 100, _stream()), "la_qgemm32_glu")
        return
    _check(lib().la_qgemm_glu(wa.fmt, a0, a1, ag, oa, b0, b1, bg, ob, F, K, x.data_ptr(), K, M, out.data_ptr(), F,
                              mode, tile, _stream()), "la_qgemm_glu")


def _time_cold(fn) -> float:
    fn()
    ts = []
    for _ in range(3):
        _cold_caches(torch.device("cuda", torch.cuda.current_device()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return sorted(ts)[1]


def glu_linear(x: torch.Tensor, ws: Sequence[QWeight], F: int, mode: int,
               bias: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """act(x Wg^T) * (x Wu^T) -> bf16 [M, F] in ONE tile-GEMM launch with the GLU activation in
    its epilogue (gate and up columns of the same index share a tile), for decode batches.  The
    autotuner times it against the unfused pair (tuned GEMM + activation kernel) once per
    32-row bucket; returns None where the fused kernel does not apply or loses."""
    if not (GLU_FUSE and TILE_GEMM and x.is_cuda and bias is None and mode in GLU_ACTS):
        return None
    M, K = x.shape
    if M > MID_MAX_M or M <= SKINNY_MAX_M:
        # prefill chunks: dequant + hipBLASLt + the activation kernel beats every fused GLU tile
        # at M >= 1024 (gemm_bs.hip's GLU mode included, profiles/r6_gemm_bs.md)
        return None
    pair = _glu_pair(ws, F)
    if pair is None:
        return None
    key = ((M + 31) // 32 * 32, K, F, mode, tuple((w.fmt, w.N) for w in ws))
    if key not in _GLU_CHOICE:
        if not GEMM_AUTOTUNE or torch.cuda.is_current_stream_capturing():
            return None
        out = torch.empty(M, F, dtype=torch.bfloat16, device=x.device)
        t_ref = _time_cold(lambda: act(linear_multi(x, ws), F, mode))
        best, best_t = None, t_ref
        cands = [6, 7, 8] if M > 128 else [7, 12, 14]
        if q32_ok([pair[0]], 9) and pair[0].fmt == pair[2].fmt:
            # (128-row tiles at M > 128 -- 107 / 105, two row tiles to fill the chip -- were timed
            # and never won: r5_glu_bench.log)
            cands += [109, 108, 104] if M > 128 else [109, 108, 107]
        if bs_ok([pair[0], pair[2]]) and pair[0].fmt == pair[2].fmt and F % 4 == 0:
            cands += [200, 203] if M > 128 else [201]
        for t in cands:
            tt = _time_cold(lambda t=t: _run_glu(x, pair, F, mode, t, out))
            if tt < best_t:
                best, best_t = t, tt
        _GLU_CHOICE[key] = best
        if os.environ.get("BENCH_DUMP_GEMM"):
            print(f"glu choice M={M} K={K} F={F} -> {best} ({best_t:.1f} us vs unfused {t_ref:.1f} us)", flush=True)
    tile = _GLU_CHOICE[key]
    if tile is None:
        return None
    out = torch.empty(M, F, dtype=torch.bfloat16, device=x.device)
    _run_glu(x, pair, F, mode, tile, out)
    return out


# ---------------------------------------------------------------------------------------
# Fused elementwise
# ---------------------------------------------------------------------------------------

def add_norm(residual: torch.Tensor, add: Optional[Partial], weight: torch.Tensor,
             bias: Optional[torch.Tensor], eps: float, mode: int = 0,
             out: Optional[torch.Tensor] = None, want_out: bool = True,
             out_f32: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """residual[T,D] (fp32, updated in place) += add;  return norm(residual)*w(+b) as bf16
    (out_f32: also written unrounded, in fp32)."""
    T, D = residual.shape
    if add is not None and (add.M != T or add.N != D):
        raise ValueError(f"add_norm: add {tuple(add.t.shape)} vs residual {T}x{D}")
    if not residual.is_cuda:
        if add is not None:
            residual += add.dense()
        if not want_out:
            return None
        x = residual
        if mode == 0:
            y = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * weight
        else:
            mu = x.mean(-1, keepdim=True)
            var = (x - mu).pow(2).mean(-1, keepdim=True)
            y = (x - mu) * torch.rsqrt(var + eps) * weight
            if bias is not None:
                y = y + bias
        if out_f32 is not None:
            out_f32.copy_(y)
        return y.to(torch.bfloat16)
    assert residual.dtype == torch.float32 and residual.is_contiguous()
    if want_out and out is None:
        out = torch.empty(T, D, dtype=torch.bfloat16, device=residual.device)
    a = add.src_args() if add is not None else (None, 0, 0, None)
    _check(lib().la_add_norm(residual.data_ptr(), a[0], a[1], a[2], a[3], int(add is not None),
                             weight.data_ptr(), _ptr(bias), _ptr(out) if want_out else None, T, D,
                             float(eps), mode, _ptr(out_f32), _stream()), "la_add_norm")
    return out if want_out else None


NORM_ROUTER = os.environ.get("LOCALAI_AMD_NORM_ROUTER", "1") == "1"


def add_norm_router(residual: torch.Tensor, add: Optional["Partial"], weight: torch.Tensor,
                    bias: Optional[torch.Tensor], eps: float, mode: int, router: torch.Tensor, topk: int,
                    renorm: bool, scale: float = 1.0, ep_base: int = 0, ep_local: int = 0):
    """add_norm + moe_router in one launch (elementwise.hip add_norm_router_kernel): returns
    (xn bf16 [T, D], ids [T, topk] int32, wts [T*topk] fp32) -- the router reads the bf16-rounded
    normed row, like moe_router on add_norm's output -- or None when the fused kernel does not
    apply (CPU, E > 64, D > 8192); the caller then runs the two ops."""
    T, D = residual.shape
    E = router.shape[0]
    if (not NORM_ROUTER or not residual.is_cuda or E > 64 or topk > min(16, E) or D % 4 or D > 8192
            or router.dtype != torch.float32 or not router.is_contiguous() or router.shape[1] != D):
        return None
    if add is not None and (add.M != T or add.N != D):
        raise ValueError(f"add_norm_router: add {tuple(add.t.shape)} vs residual {T}x{D}")
    assert residual.dtype == torch.float32 and residual.is_contiguous()
    out = torch.empty(T, D, dtype=torch.bfloat16, device=residual.device)
    ids = torch.empty(T, topk, dtype=torch.int32, device=residual.device)
    wts = torch.empty(T * topk, dtype=torch.float32, device=residual.device)
    a = add.src_args() if add is not None else (None, 0, 0, None)
    _check(lib().la_add_norm_router(residual.data_ptr(), a[0], a[1], a[2], a[3], int(add is not None),
                                    weight.data_ptr(), _ptr(bias), out.data_ptr(), T, D, float(eps), mode,
                                    router.data_ptr(), E, topk, int(renorm), float(scale), ep_base,
                                    ep_local or E, ids.data_ptr(), wts.data_ptr(), _stream()), "la_add_norm_router")
    return out, ids, wts


def rope_cos_sin(max_pos: int, rot_dim: int, theta: float, device, freq_scale: float = 1.0,
                 freq_factors: Optional[torch.Tensor] = None, rope_type: str = "none",
                 yarn: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, rot/2, 2] (cos, sin) table, fp32, computed in float64 on the host."""
    half = rot_dim // 2
    inv = 1.0 / (theta ** (np.arange(0, half, dtype=np.float64) * 2.0 / rot_dim))
    if freq_factors is not None:
        inv = inv / freq_factors.detach().cpu().double().numpy()[:half]
    mscale = 1.0
    if rope_type == "yarn" and yarn:
        # YaRN (ggml rope_yarn): blend interpolated/extrapolated frequencies by ramp
        orig = yarn.get("orig_ctx", 4096)
        bf, bs = yarn.get("beta_fast", 32.0), yarn.get("beta_slow", 1.0)
        ext = yarn.get("ext_factor", 1.0)
        def corr_dim(nrot):
            return rot_dim * math.log(orig / (nrot * 2 * math.pi)) / (2 * math.log(theta))
        lo = max(0.0, math.floor(corr_dim(bf)))
        hi = min(rot_dim - 1.0, math.ceil(corr_dim(bs)))
        i = np.arange(half, dtype=np.float64)
        ramp = np.clip((i - lo) / max(0.001, hi - lo), 0, 1)
        mix = (1 - ramp) * ext
        inv = inv * freq_scale * (1 - mix) + inv * mix
        mscale = yarn.get("attn_factor", 1.0) * (1.0 + 0.1 * math.log(1.0 / freq_scale)) if freq_scale < 1 else \
            yarn.get("attn_factor", 1.0)
    else:
        inv = inv * freq_scale
    pos = np.arange(max_pos, dtype=np.float64)
    ang = np.outer(pos, inv)
    cs = np.stack([np.cos(ang) * mscale, np.sin(ang) * mscale], -1).astype(np.float32)
    return torch.from_numpy(cs).to(device)


def rope_kv(qkv: Partial, pos: torch.Tensor, slots: Optional[torch.Tensor], cos_sin: torch.Tensor,
            Hq: int, Hkv: int, Dh: int, rot: int, mode: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
            block_size: int, q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rotate q,k; write k,v into the paged cache at `slots`; return q [T,Hq,Dh] bf16."""
    T = qkv.M
    W = (Hq + 2 * Hkv) * Dh
    if qkv.N != W:
        raise ValueError(f"rope_kv: qkv width {qkv.N} != {W}")
    if not qkv.t.is_cuda:
        x = qkv.dense().view(T, Hq + 2 * Hkv, Dh)
        cs = cos_sin[pos.long()]  # [T, rot/2, 2]
        c, s = cs[..., 0], cs[..., 1]

        def rot_fn(h):
            h = h.clone()
            if mode == 0:
                x0, x1 = h[..., 0:rot:2].clone(), h[..., 1:rot:2].clone()
                h[..., 0:rot:2] = x0 * c[:, None] - x1 * s[:, None]
                h[..., 1:rot:2] = x0 * s[:, None] + x1 * c[:, None]
            else:
                half = rot // 2
                x0, x1 = h[..., :half].clone(), h[..., half:rot].clone()
                h[..., :half] = x0 * c[:, None] - x1 * s[:, None]
                h[..., half:rot] = x0 * s[:, None] + x1 * c[:, None]
            return h
        q = rot_fn(x[:, :Hq]).to(torch.bfloat16)
        k = rot_fn(x[:, Hq:Hq + Hkv]).to(k_cache.dtype)
        v = x[:, Hq + Hkv:].to(v_cache.dtype)
        if slots is not None:
            sl = slots.long()
            ok = sl >= 0
            blk, off = sl[ok] // block_size, sl[ok] % block_size
            k_cache[blk, :, off] = k[ok]
            v_cache[blk, :, off // 8, :, off % 8] = v[ok]
        if q_out is not None:
            q_out.copy_(q)
            return q_out
        return q
    if q_out is None:
        q_out = torch.empty(T, Hq, Dh, dtype=torch.bfloat16, device=qkv.t.device)
    a = qkv.src_args()
    _check(lib().la_rope_kv(a[0], a[1], a[2], a[3], pos.data_ptr(), _ptr(slots), cos_sin.data_ptr(), T, Hq, Hkv,
                            Dh, rot, mode, q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_size,
                            _stream()), "la_rope_kv")
    return q_out


ACT_SWIGLU, ACT_GELU, ACT_GELU_QUICK, ACT_GEGLU = 0, 1, 2, 3
GLU_ACTS = (ACT_SWIGLU, ACT_GEGLU)  # gate|up sources of width 2F


def act(src: Partial, F: int, mode: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    T = src.M
    if not src.t.is_cuda:
        x = src.dense()
        if mode == ACT_SWIGLU:
            y = torch.nn.functional.silu(x[:, :F]) * x[:, F:2 * F]
        elif mode == ACT_GEGLU:
            y = torch.nn.functional.gelu(x[:, :F], approximate="tanh") * x[:, F:2 * F]
        elif mode == ACT_GELU:
            y = torch.nn.functional.gelu(x, approximate="tanh")
        else:
            y = x * torch.sigmoid(1.702 * x)
        return y.to(torch.bfloat16)
    if out is None:
        out = torch.empty(T, F, dtype=torch.bfloat16, device=src.t.device)
    a = src.src_args()
    _check(lib().la_act(a[0], a[1], a[2], a[3], out.data_ptr(), T, F, mode, _stream()), "la_act")
    return out


def act_linear(src: Partial, F: int, mode: int, w: QWeight) -> Partial:
    """down(act(gate|up)).  On the decode GEMV path (M <= GEMV_MAX_M, fp32 slab source) the
    activation is computed inside the down GEMV's activation prologue -- no activation launch
    and no bf16 round trip; otherwise act() then linear()."""
    M = src.M
    width = 2 * F if mode in GLU_ACTS else F
    if (src.t.is_cuda and src.S >= 1 and src.S <= 16 and GEMV_DP4 and M <= GEMV_MAX_M and w.gemv_ok
            and w.K == F and src.N == width):
        S = _gemv_splits([w], w.K, M)
        out = torch.empty(S, M, w.N, dtype=torch.float32, device=src.t.device)
        gemv_dp4(None, [w], S, out, act_src=src, act_mode=mode)
        return Partial(out)
    return linear(act(src, F, mode), w)


def reduce(src: Partial, dtype=torch.float32, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum of the split-K slabs (+ bias) as one dense [M, N] matrix (into `out`, a contiguous
    [M, N] tensor of `dtype`, when given)."""
    if out is not None:
        dtype = out.dtype
        assert out.is_contiguous() and tuple(out.shape) == (src.M, src.N)
    if not src.t.is_cuda:
        d = src.dense().to(dtype)
        if out is None:
            return d
        out.copy_(d)
        return out
    T, N = src.M, src.N
    if out is None:
        out = torch.empty(T, N, dtype=dtype, device=src.t.device)
    a = src.src_args()
    f32 = out.data_ptr() if dtype == torch.float32 else None
    b16 = out.data_ptr() if dtype == torch.bfloat16 else None
    _check(lib().la_reduce_slabs(a[0], a[1], a[2], a[3], T, N, f32, b16, _stream()), "la_reduce_slabs")
    return out


def embed(tokens: torch.Tensor, w: QWeight, scale: float = 1.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    T = tokens.shape[0]
    if not tokens.is_cuda:
        return w.dequant_f32()[tokens.long()] * scale
    if out is None:
        out = torch.empty(T, w.K, dtype=torch.float32, device=tokens.device)
    assert tokens.dtype == torch.int32
    _check(lib().la_embed(w.fmt, *w.ptrs(), w.N, w.K, tokens.data_ptr(), T, out.data_ptr(), float(scale),
                          _stream()), "la_embed")
    return out


def gather_rows(src: torch.Tensor, idx: torch.Tensor, fill: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[t] = src[idx[t]] if idx[t] >= 0 else fill: one launch (elementwise.hip gather_rows_kernel).
    src [R, C] contiguous, idx int64 [T] on the same device, fill [C] (needed when idx has -1s)."""
    T, C = idx.shape[0], src.shape[1]
    if not src.is_cuda:
        out = src[idx.clamp(min=0)]
        if fill is not None:
            out[idx < 0] = fill.to(out.dtype)
        return out
    assert src.is_contiguous() and idx.dtype == torch.int64 and idx.device == src.device
    out = torch.empty(T, C, dtype=src.dtype, device=src.device)
    if fill is not None:
        fill = fill.to(src.dtype).contiguous()
    _check(lib().la_gather_rows(src.data_ptr(), idx.data_ptr(), T, _ptr(fill), out.data_ptr(),
                                C * src.element_size(), _stream()), "la_gather_rows")
    return out


# ---------------------------------------------------------------------------------------
# Attention
# ---------------------------------------------------------------------------------------

DEC_TARGET_WAVES = 2048  # ~16 waves per CU over 256 CUs
# (sequence, kv head) pairs for which attn_decode runs single-wave workgroups: 2048 of them
# (decode batch 256 x 8 kv heads) are resident at once at 2 waves per SIMD, so every workgroup's
# latency chain (seq_len -> block table -> first K/V tile) starts in ONE residency round, where
# 4-wave workgroups go through 4 rounds.  Measured on MI355X (scripts/attn_bench.py, KV cycled
# through 8 layers' worth of HBM): B=256 x L=384 72.6 vs 74.9 us, B=256 x L=256 equal, but
# B=128 (two partitions per sequence) 50.6 vs 40.2 us and B=512 (two rounds) 119.7 vs 114.0 us,
# hence the window
DEC_NW1_MIN = int(os.environ.get("LOCALAI_AMD_DEC_NW1_MIN", "2048"))
DEC_NW1_MAX = 2048


def decode_waves(B: int, Hkv: int) -> int:
    """Waves per attn_decode workgroup (1 or 4) for a batch of B sequences."""
    return 1 if DEC_NW1_MIN <= B * Hkv <= max(DEC_NW1_MAX, DEC_NW1_MIN) else 4


# B * Hkv up to this: short sequences are split over the grid's partitions too (32-key
# granularity) instead of running as one partition -- a handful of workgroups cannot hide the
# KV load latency at batch 1 (attn_decode's one_part rule, nw bit 8)
DEC_SPLIT_SHORT = int(os.environ.get("LOCALAI_AMD_DEC_SPLIT_SHORT", "0"))


def _dec_split_short(B: int, Hkv: int) -> bool:
    return B * Hkv <= DEC_SPLIT_SHORT


def decode_partitions(B: int, Hkv: int, max_len: int, block_size: int = 32) -> Tuple[int, int]:
    """Split-KV partitioning for attn_decode: (P, PS).  Enough partitions to put ~16 waves on
    every CU; each workgroup (decode_waves waves) covers PS keys (multiple of 128 -- of 32 for
    the few-sequence split -- at most 2048 pages so the partition's block-table slice fits the
    kernel's LDS stage)."""
    max_len = max(1, max_len)
    nw = decode_waves(B, Hkv)
    gran = max(32, block_size) if _dec_split_short(B, Hkv) else 128
    P = max(1, min(-(-DEC_TARGET_WAVES // (B * Hkv * nw)), -(-max_len // gran), 64))
    P = max(P, -(-max_len // (2048 * block_size)))
    PS = -(-(-(-max_len // P)) // gran) * gran
    P = -(-max_len // PS)
    return P, PS


def _dec_nw(B: int, Hkv: int) -> int:
    return decode_waves(B, Hkv) | (256 if _dec_split_short(B, Hkv) else 0)


def decode_workspace(B: int, Hq: int, Hkv: int, Dh: int, max_len: int, device, block_size: int = 32):
    """Persistent buffers for attn_decode (split-KV partials + self-resetting merge tickets)."""
    P, _ = decode_partitions(B, Hkv, max_len, block_size)
    return (torch.empty(max(1, B * Hq * P * Dh), dtype=torch.float32, device=device),
            torch.empty(max(1, B * Hq * P * 2), dtype=torch.float32, device=device),
            torch.zeros(max(1, B * Hkv), dtype=torch.int32, device=device))


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                seq_lens: torch.Tensor, scale: float, max_seq_len: int, out: Optional[torch.Tensor] = None,
                workspace: Optional[Tuple[torch.Tensor, ...]] = None, softcap: float = 0.0,
                window: int = 0) -> torch.Tensor:
    """q [B,Hq,Dh] bf16; K cache [nblk,Hkv,BS,Dh]; V cache (grouped-transposed pages)
    [nblk,Hkv,BS/8,Dh,8]; block_tables [B,maxb] i32; seq_lens [B] i32.  softcap > 0: scores
    softcap * tanh(s / softcap); window > 0: only the last `window` keys are attended (Gemma-2)."""
    B, Hq, Dh = q.shape
    nblk, Hkv, BS, Dh2 = k_cache.shape
    if Dh2 != Dh or Hq % Hkv or tuple(v_cache.shape) != (nblk, Hkv, BS // 8, Dh, 8):
        raise ValueError("attn_decode: head/cache shape mismatch")
    if not q.is_cuda:
        return _attn_ref_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, softcap, window)
    P, PS = decode_partitions(B, Hkv, max_seq_len, BS)
    if out is None:
        out = torch.empty(B, Hq, Dh, dtype=torch.bfloat16, device=q.device)
    if (workspace is None or len(workspace) < 3 or workspace[0].numel() < B * Hq * P * Dh
            or workspace[1].numel() < B * Hq * P * 2 or workspace[2].numel() < B * Hkv):
        workspace = decode_workspace(B, Hq, Hkv, Dh, max_seq_len, q.device, BS)
    po, pml, tk = workspace[:3]
    _check(lib().la_attn_decode(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
                                block_tables.shape[1], seq_lens.data_ptr(), B, Hq, Hkv, Dh, BS, float(scale), P, PS,
                                out.data_ptr(), po.data_ptr(), pml.data_ptr(), tk.data_ptr(), None, 0, 0, None, None,
                                None, None, float(softcap), int(window), _dec_nw(B, Hkv), _stream()),
           "la_attn_decode")
    return out


# Off by default: measured on MI355X (Llama-3-8B Q4_K_M, engine bench) the fused launch is not
# faster -- C=1 435.5 vs 440.4 tok/s, C=256 26.43k vs 26.55k -- because the q|k|v slab loads move
# onto the attention kernel's critical path instead of disappearing with the rope_kv launch.
FUSED_DECODE_ROPE = os.environ.get("LOCALAI_AMD_FUSED_ROPE", "0") == "1"


def attn_decode_rope(qkv: Partial, pos: torch.Tensor, slots: torch.Tensor, cos_sin: torch.Tensor, Hq: int,
                     Hkv: int, Dh: int, rot: int, mode: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
                     block_tables: torch.Tensor, seq_lens: torch.Tensor, scale: float, max_seq_len: int,
                     out: Optional[torch.Tensor] = None,
                     workspace: Optional[Tuple[torch.Tensor, ...]] = None, softcap: float = 0.0,
                     window: int = 0) -> torch.Tensor:
    """Decode step attention with the step's RoPE + paged KV append fused into the attention
    kernel (one launch instead of rope_kv + attn_decode).  Same numerics as the two-kernel path
    (q/k rotated in fp32, rounded to bf16).  Falls back to rope_kv + attn_decode for NEOX /
    partial rotary, Dh not a multiple of 32, or CPU tensors."""
    T = qkv.M
    nblk, _, BS, _ = k_cache.shape
    fusable = (FUSED_DECODE_ROPE and qkv.t.is_cuda and mode == 0 and rot == Dh and Dh % 32 == 0
               and k_cache.dtype == torch.bfloat16 and v_cache.dtype == torch.bfloat16
               and qkv.N == (Hq + 2 * Hkv) * Dh and (qkv.S >= 1 or qkv.t.dtype == torch.bfloat16)
               and tuple(cos_sin.shape[1:]) == (Dh // 2, 2))
    if not fusable:
        q = rope_kv(qkv, pos, slots, cos_sin, Hq, Hkv, Dh, rot, mode, k_cache, v_cache, BS)
        return attn_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, max_seq_len, out=out,
                           workspace=workspace, softcap=softcap, window=window)
    if Hq % Hkv or tuple(v_cache.shape) != (nblk, Hkv, BS // 8, Dh, 8) or k_cache.shape[3] != Dh:
        raise ValueError("attn_decode_rope: head/cache shape mismatch")
    P, PS = decode_partitions(T, Hkv, max_seq_len, BS)
    if out is None:
        out = torch.empty(T, Hq, Dh, dtype=torch.bfloat16, device=qkv.t.device)
    if (workspace is None or len(workspace) < 3 or workspace[0].numel() < T * Hq * P * Dh
            or workspace[1].numel() < T * Hq * P * 2 or workspace[2].numel() < T * Hkv):
        workspace = decode_workspace(T, Hq, Hkv, Dh, max_seq_len, qkv.t.device, BS)
    po, pml, tk = workspace[:3]
    a = qkv.src_args()
    _check(lib().la_attn_decode(None, k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
                                block_tables.shape[1], seq_lens.data_ptr(), T, Hq, Hkv, Dh, BS, float(scale), P, PS,
                                out.data_ptr(), po.data_ptr(), pml.data_ptr(), tk.data_ptr(), a[0], a[1], a[2], a[3],
                                pos.data_ptr(), slots.data_ptr(), cos_sin.data_ptr(), float(softcap), int(window),
                                _dec_nw(T, Hkv), _stream()),
           "la_attn_decode(rope)")
    return out


def v_pages(nblk: int, Hkv: int, BS: int, Dh: int, dtype=torch.bfloat16, device=None) -> torch.Tensor:
    """An empty V cache in the kernels' layout: [nblk, Hkv, BS/8, Dh, 8]."""
    return torch.zeros(nblk, Hkv, BS // 8, Dh, 8, dtype=dtype, device=device)


def v_from_rows(v: torch.Tensor) -> torch.Tensor:
    """[nblk, Hkv, BS, Dh] (key-major pages) -> the V cache layout [nblk, Hkv, BS/8, Dh, 8]."""
    n, h, bs, d = v.shape
    return v.view(n, h, bs // 8, 8, d).transpose(3, 4).contiguous()


def _gather_kv(cache, bt_row, L, transposed=False):
    """-> [Hkv, L, Dh] from K pages [nblk,Hkv,BS,Dh] or V pages [nblk,Hkv,BS/8,Dh,8]."""
    if transposed:
        n, h, g, d, e = cache.shape
        cache = cache.transpose(3, 4).reshape(n, h, g * e, d)
    BS = cache.shape[2]
    nb = (L + BS - 1) // BS
    blocks = cache[bt_row[:nb].long()]                  # [nb, Hkv, BS, Dh]
    return blocks.permute(1, 0, 2, 3).reshape(cache.shape[1], nb * BS, cache.shape[3])[:, :L]


def _softcap_window(s, softcap, window, qpos, kpos):
    """Gemma-2 score transforms of the CPU references: soft-capping, then the sliding window."""
    if softcap > 0:
        s = softcap * torch.tanh(s / softcap)
    if window > 0:
        s = s.masked_fill(qpos - kpos >= window, float("-inf"))
    return s


def _attn_ref_decode(q, kc, vc, bt, sl, scale, softcap=0.0, window=0):
    B, Hq, Dh = q.shape
    Hkv = kc.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    for b in range(B):
        L = int(sl[b])
        k = _gather_kv(kc, bt[b], L).float()
        v = _gather_kv(vc, bt[b], L, transposed=True).float()
        qq = q[b].float().view(Hkv, G, Dh)
        s = torch.einsum("hgd,hld->hgl", qq, k) * scale
        s = _softcap_window(s, softcap, window, torch.tensor(L - 1), torch.arange(L))
        p = torch.softmax(s, -1)
        out[b] = torch.einsum("hgl,hld->hgd", p, v).reshape(Hq, Dh).to(q.dtype)
    return out


PF_QT = 64


def prefill_tiles(q_lens: Sequence[int], device) -> torch.Tensor:
    tiles = []
    for s, ql in enumerate(q_lens):
        for r in range(0, ql, PF_QT):
            tiles.append((s, r))
    return torch.tensor(tiles, dtype=torch.int32, device=device).view(-1, 2)


def attn_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, cu_q: torch.Tensor,
                 ctx_lens: torch.Tensor, block_tables: torch.Tensor, scale: float,
                 tiles: Optional[torch.Tensor] = None, q_lens: Optional[Sequence[int]] = None,
                 out: Optional[torch.Tensor] = None, softcap: float = 0.0, window: int = 0) -> torch.Tensor:
    """Causal attention for new tokens. q [T,Hq,Dh]; cu_q [nseq+1]; ctx_lens [nseq] (cached+new)."""
    T, Hq, Dh = q.shape
    Hkv = k_cache.shape[1]
    if not q.is_cuda:
        return _attn_ref_prefill(q, k_cache, v_cache, cu_q, ctx_lens, block_tables, scale, softcap, window)
    if tiles is None:
        cq = cu_q.cpu().tolist()
        tiles = prefill_tiles([cq[i + 1] - cq[i] for i in range(len(cq) - 1)], q.device)
    if out is None:
        out = torch.empty(T, Hq, Dh, dtype=torch.bfloat16, device=q.device)
    _check(lib().la_attn_prefill(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), tiles.data_ptr(),
                                 tiles.shape[0], cu_q.data_ptr(), ctx_lens.data_ptr(), block_tables.data_ptr(),
                                 block_tables.shape[1], Hq, Hkv, Dh, k_cache.shape[2], float(scale),
                                 out.data_ptr(), float(softcap), int(window), _stream()), "la_attn_prefill")
    return out


_DENSE_META: Dict[tuple, tuple] = {}


def attn_dense(qkv: torch.Tensor, n: int, L: int, H: int, scale: Optional[float] = None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Non-causal self-attention of n sequences of L tokens, read in place from a fused q|k|v
    projection output [n * L, 3 * D] (bf16; D = H * Dh): the MFMA flash-attention kernel of
    la_attn_prefill in its dense mode (vision towers).  Returns [n * L, D] bf16."""
    T, W = qkv.shape
    D = W // 3
    Dh = D // H
    if scale is None:
        scale = Dh ** -0.5
    if not qkv.is_cuda:
        q, k, v = qkv.float().view(n, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
        o = torch.softmax(q @ k.transpose(-1, -2) * scale, -1) @ v
        return o.transpose(1, 2).reshape(T, D).to(qkv.dtype)
    if qkv.dtype != torch.bfloat16 or not qkv.is_contiguous() or T != n * L or W != 3 * D:
        raise ValueError("attn_dense: qkv must be a contiguous bf16 [n * L, 3 * D] matrix")
    key = (n, L, qkv.device)
    meta = _DENSE_META.get(key)
    if meta is None:
        cu = torch.arange(0, (n + 1) * L, L, dtype=torch.int32, device=qkv.device)
        meta = _DENSE_META[key] = (cu, prefill_tiles([L] * n, qkv.device))
    cu, tiles = meta
    if out is None:
        out = torch.empty(T, D, dtype=torch.bfloat16, device=qkv.device)
    base = qkv.data_ptr()
    _check(lib().la_attn_dense(base, W, base + 2 * D, W, base + 4 * D, W, out.data_ptr(), D, tiles.data_ptr(),
                               tiles.shape[0], cu.data_ptr(), H, H, Dh, float(scale), _stream()), "la_attn_dense")
    return out


def _attn_ref_prefill(q, kc, vc, cu_q, ctx_lens, bt, scale, softcap=0.0, window=0):
    T, Hq, Dh = q.shape
    Hkv = kc.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    cq = cu_q.tolist()
    for s in range(len(cq) - 1):
        a, b = cq[s], cq[s + 1]
        ql = b - a
        if ql == 0:
            continue
        L = int(ctx_lens[s])
        k = _gather_kv(kc, bt[s], L).float().repeat_interleave(G, 0)   # [Hq, L, Dh]
        v = _gather_kv(vc, bt[s], L, transposed=True).float().repeat_interleave(G, 0)
        qq = q[a:b].float().transpose(0, 1)                              # [Hq, ql, Dh]
        sc = torch.einsum("hqd,hld->hql", qq, k) * scale
        qpos = torch.arange(L - ql, L).view(-1, 1)
        kpos = torch.arange(L).view(1, -1)
        sc = _softcap_window(sc, softcap, window, qpos, kpos)
        sc = sc.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(sc, -1)
        out[a:b] = torch.einsum("hql,hld->hqd", p, v).transpose(0, 1).to(q.dtype)
    return out


# ---------------------------------------------------------------------------------------
# Sampling
# ---------------------------------------------------------------------------------------

SAMPLE_ROW_DTYPE = np.dtype([("temp", "<f4"), ("top_p", "<f4"), ("min_p", "<f4"), ("typical_p", "<f4"),
                             ("tfs_z", "<f4"), ("tau", "<f4"), ("eta", "<f4"), ("top_k", "<i4"),
                             ("mirostat", "<i4"), ("pad", "<i4"), ("seed", "<u8"), ("counter", "<u8")])


def sample(logits: torch.Tensor, params: np.ndarray, mu: Optional[torch.Tensor] = None,
           params_dev: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits [B, V] f32; params: structured array (SAMPLE_ROW_DTYPE) of length B."""
    B, V = logits.shape
    assert params.dtype == SAMPLE_ROW_DTYPE and len(params) == B
    if not logits.is_cuda:
        return sample_ref(logits, params, mu)
    if logits.dtype != torch.float32 or logits.stride(1) != 1:
        raise ValueError("sample: logits must be f32 with unit column stride")
    if params_dev is None:
        params_dev = torch.from_numpy(params.view(np.uint8).copy()).to(logits.device, non_blocking=True)
    if mu is None:
        mu = torch.zeros(B, dtype=torch.float32, device=logits.device)
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    _check(lib().la_sample(logits.data_ptr(), logits.stride(0), B, V, params_dev.data_ptr(), mu.data_ptr(),
                           out.data_ptr(), None, _stream()), "la_sample")
    return out


def sample_ref(logits: torch.Tensor, params: np.ndarray, mu: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Host reference of the sampler chain (same semantics, torch RNG)."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        p = params[b]
        l = logits[b].float().cpu()
        if p["temp"] <= 0:
            out[b] = int(torch.argmax(l))
            continue
        g = torch.Generator().manual_seed(int(p["seed"]) ^ int(p["counter"]))
        if p["mirostat"] == 2:
            pr = torch.softmax(l / float(p["temp"]), -1)
            m = float(mu[b]) if mu is not None else 2 * float(p["tau"])
            keep = pr >= 2.0 ** (-m)
            keep[torch.argmax(pr)] = True
            q = torch.where(keep, pr, torch.zeros_like(pr))
            q = q / q.sum()
            t = int(torch.multinomial(q, 1, generator=g))
            if mu is not None:
                mu[b] = m - float(p["eta"]) * (-math.log2(float(q[t])) - float(p["tau"]))
            out[b] = t
            continue
        vals, idx = torch.sort(l, descending=True, stable=True)
        k = int(p["top_k"])
        if 0 < k < V:
            vals, idx = vals[:k], idx[:k]
        pr = torch.softmax(vals, -1)
        n = len(vals)
        if p["top_p"] < 1:
            cs = torch.cumsum(pr, 0)
            hit = torch.nonzero(cs >= float(p["top_p"]))
            if len(hit):
                n = min(n, int(hit[0]) + 1)
        if p["min_p"] > 0:
            keepm = int((vals >= vals[0] + math.log(float(p["min_p"]))).sum())
            n = min(n, max(1, keepm))
        vals, idx = vals[:n], idx[:n]
        q = torch.softmax(vals / float(p["temp"]), -1)
        out[b] = int(idx[int(torch.multinomial(q, 1, generator=g))])
    return out


def logit_bias(logits: torch.Tensor, rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor,
               count: torch.Tensor):
    """In place: logits[rows[i], cols[i]] += vals[i] for i < count[0] (graph-capturable: the
    entry count lives on the device)."""
    cap = rows.shape[0]
    if not logits.is_cuda:
        n = int(count[0])
        logits.index_put_((rows[:n].long(), cols[:n].long()), vals[:n].to(logits.dtype), accumulate=True)
        return logits
    _check(lib().la_logit_bias(logits.data_ptr(), logits.stride(0), rows.data_ptr(), cols.data_ptr(),
                               vals.data_ptr(), count.data_ptr(), cap, _stream()), "la_logit_bias")
    return logits


def decode_advance(next_tok, tok, pos, lens, slots, bt, block_size: int, hist, step, prm_dev):
    """Feed sampled tokens back as the next decode inputs (see csrc/decode_loop.hip)."""
    B = tok.shape[0]
    if not tok.is_cuda:
        s = int(step[0])
        if s < hist.shape[0]:
            hist[s] = next_tok
        live = slots >= 0
        tok[live] = next_tok[live]
        pos[live] += 1
        lens[live] = pos[live] + 1
        p = pos[live].long()
        slots[live] = (bt[live, p // block_size] * block_size + (p % block_size)).to(slots.dtype)
        rows = prm_dev.numpy().view(SAMPLE_ROW_DTYPE)
        rows["counter"][live.numpy()] += 1
        step[0] = s + 1
        return
    _check(lib().la_decode_advance(next_tok.data_ptr(), tok.data_ptr(), pos.data_ptr(), lens.data_ptr(),
                                   slots.data_ptr(), bt.data_ptr(), bt.stride(0), block_size, B, hist.data_ptr(),
                                   hist.shape[0], step.data_ptr(), prm_dev.data_ptr(), _stream()),
           "la_decode_advance")


# ---------------------------------------------------------------------------------------
# Mixture of experts (decode-sized batches; csrc/moe.hip)
# ---------------------------------------------------------------------------------------

class MoEWeights:
    """E experts of one projection (same format / shape) + their QW descriptors on the device."""

    def __init__(self, experts: Sequence[QWeight]):
        if not experts or len({(w.fmt, w.N, w.K) for w in experts}) != 1:
            raise ValueError("MoEWeights: experts must share format and shape")
        self.experts = list(experts)
        self.E, self.N, self.K, self.fmt = len(experts), experts[0].N, experts[0].K, experts[0].fmt
        self.desc = None
        p0 = experts[0].planes[0]
        if p0 is not None and p0.device.type == "cuda":
            dev = p0.device
            qw = np.zeros(self.E, dtype=[("p", "<u8", 4), ("N", "<i4"), ("K", "<i4")])
            assert qw.dtype.itemsize == lib().la_qw_size()
            for e, w in enumerate(experts):
                qw[e]["p"] = [_ptr(p) or 0 for p in w.planes]
                qw[e]["N"], qw[e]["K"] = w.N, w.K
            self.desc = torch.from_numpy(qw.view(np.uint8).copy()).to(dev)
        self._desc32 = None

    def desc32(self) -> torch.Tensor:
        """Descriptors for the 32x32x16 grouped GEMM (la_moe32): {codes, aux, blocked scale
        plane, -} per expert; the scale planes are built on first use (0.125 B per weight)."""
        if self._desc32 is None:
            qw = np.zeros(self.E, dtype=[("p", "<u8", 4), ("N", "<i4"), ("K", "<i4")])
            for e, w in enumerate(self.experts):
                p0, p1, g = w.tile_planes()
                qw[e]["p"] = [p0 or 0, p1 or 0, g or 0, 0]
                qw[e]["N"], qw[e]["K"] = w.N, w.K
            self._desc32 = torch.from_numpy(qw.view(np.uint8).copy()).to(self.desc.device)
        return self._desc32


def moe_router(xn: torch.Tensor, router: torch.Tensor, topk: int, renorm: bool, scale: float = 1.0,
               ep_base: int = 0, ep_local: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused router for decode batches: xn [T, D] bf16, router [E, D] fp32 -> (ids [T, topk] int32,
    weights [T*topk] fp32): softmax over E, top-k by probability, optional renormalisation and
    scale; under expert parallelism ids are local (ep_base..ep_base+ep_local-1 -> 0..) and other
    ranks' experts map to ep_local."""
    T, D = xn.shape
    E = router.shape[0]
    local = ep_local or E
    if not xn.is_cuda:
        p = torch.softmax(xn.float() @ router.t(), -1)
        w, idx = torch.topk(p, topk, -1)
        if renorm:
            w = w / w.sum(-1, keepdim=True)
        loc = idx - ep_base
        ids = torch.where((loc >= 0) & (loc < local), loc, torch.full_like(loc, local)).to(torch.int32)
        return ids, (w * scale).reshape(-1).float()
    assert xn.dtype == torch.bfloat16 and xn.stride(-1) == 1 and router.dtype == torch.float32
    assert router.is_contiguous() and router.shape[1] == D and D % 8 == 0 and E <= 256 and topk <= min(16, E)
    ids = torch.empty(T, topk, dtype=torch.int32, device=xn.device)
    wts = torch.empty(T * topk, dtype=torch.float32, device=xn.device)
    _check(lib().la_moe_router(xn.data_ptr(), xn.stride(0), router.data_ptr(), E, D, T, topk, int(renorm),
                               float(scale), ep_base, local, ids.data_ptr(), wts.data_ptr(), _stream()),
           "la_moe_router")
    return ids, wts


def moe_route(ids: torch.Tensor, E: int, order: Optional[torch.Tensor] = None, off: Optional[torch.Tensor] = None):
    """ids [T, topk] int32 -> (order [T*topk] pair ids grouped by expert, off [E+1])."""
    T, topk = ids.shape
    if order is None:
        order = torch.empty(T * topk, dtype=torch.int32, device=ids.device)
    if off is None:
        off = torch.empty(E + 1, dtype=torch.int32, device=ids.device)
    if not ids.is_cuda:
        flat = ids.reshape(-1).long()
        perm = torch.sort(flat, stable=True).indices
        order.copy_(perm.to(torch.int32))
        cnt = torch.bincount(flat, minlength=E)
        off.copy_(torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)]).to(torch.int32))
        return order, off
    ids = ids.contiguous().to(torch.int32)
    _check(lib().la_moe_route(ids.data_ptr(), T, topk, E, order.data_ptr(), off.data_ptr(), _stream()), "la_moe_route")
    return order, off


def moe_linear(x: torch.Tensor, mw: MoEWeights, order: torch.Tensor, off: torch.Tensor, topk: int, T: int,
               down: bool = False, wts: Optional[torch.Tensor] = None, zero: bool = False) -> Partial:
    """Grouped expert GEMM.  gate/up (down=False): x [T, K] -> Partial [S, T*topk, N] (row = pair).
    down (down=True): x [T*topk, K] (row = pair) -> Partial [S*topk, T, N], each slab scaled by
    the routing weight, so summing the slabs performs the weighted top-k combine.  Pairs routed to
    an expert id >= mw.E (expert parallelism: another rank's expert) are not computed; with
    zero=True their down-projection rows read as 0."""
    if not x.is_cuda:
        P = T * topk
        flat_e = torch.full((P,), -1, dtype=torch.long)
        offs = off.tolist()
        for e in range(mw.E):
            flat_e[order[offs[e]:offs[e + 1]].long()] = e
        if down:
            out = torch.zeros(topk, T, mw.N)
            for p in range(P):
                t, slot = divmod(p, topk)
                if flat_e[p] < 0:
                    continue
                out[slot, t] = (x[p].float() @ mw.experts[int(flat_e[p])].dequant_f32().t()) * float(wts[p])
        else:
            out = torch.zeros(1, P, mw.N)
            for p in range(P):
                if flat_e[p] >= 0:
                    out[0, p] = x[p // topk].float() @ mw.experts[int(flat_e[p])].dequant_f32().t()
        return Partial(out)
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("moe_linear: x must be contiguous bf16")
    maxM = T  # a token picks an expert at most once; above 64 rows the launch adds row chunks
    S = pick_splits(mw.N, mw.K, maxM)
    nsb = mw.K // 256
    while nsb % S:
        S -= 1
    P = T * topk
    if down:
        alloc = torch.zeros if zero else torch.empty
        out = alloc(S * topk, T, mw.N, dtype=torch.float32, device=x.device)
        slab = T * mw.N
    else:
        out = torch.empty(S, P, mw.N, dtype=torch.float32, device=x.device)
        slab = P * mw.N
    _check(lib().la_moe_gemm(mw.fmt, 1 if down else 0, mw.desc.data_ptr(), mw.N, mw.K, mw.E, order.data_ptr(),
                             off.data_ptr(), topk, x.data_ptr(), x.shape[1], maxM, S,
                             _ptr(wts) if down else None, out.data_ptr(), mw.N, slab, T, _stream()), "la_moe_gemm")
    return Partial(out)


# Grouped expert GEMMs on the 32x32x16 tile (gemm_q32.hip moe32_kernel) for batches of at least
# MOE32_MIN_T tokens: gate|up with the SwiGLU fused (bf16 h in grouped row order), then the
# routing-weighted down projection.  Variant ids: gemm_q32.hip moe32_var.
MOE32 = os.environ.get("LOCALAI_AMD_MOE32", "1") == "1"
# Variant by batch (scripts/moe_bench.py, Mixtral-8x7B shapes, gpurun_out/r5_moe32_bench.log):
# T = 64: 32-row tiles, 4 workgroups per CU (var 9) 156 + 86 us vs the 16-column kernel's
# 285 + 9 (act) + 143; T = 128 / 256: 64-row tiles in 8-wave workgroups (var 4) 180 + 91 /
# 291 + 162 us vs 276 + 15 + 145 / 470 + 16 + 255.
# T = 16 / 24 / 32: var 9 232 / 234 / 237 us vs 266 / 315 / 317; T = 8: 221 vs 212
# (gpurun_out/r5_moe_small.log)
MOE32_MIN_T = int(os.environ.get("LOCALAI_AMD_MOE32_MIN_T", "12"))
MOE32_SMALL_T = 48     # below: var 9 (32-row tiles); from here: var 17 (64-row chunks, live row blocks)
MOE32_LIVE_BIG_T = 192  # from here: var 19 (one 128-row chunk per expert at top-2 of 8)
MOE32_VAR_GLU = int(os.environ.get("LOCALAI_AMD_MOE32_VAR_GLU", "-1"))     # -1: by batch
MOE32_VAR_DOWN = int(os.environ.get("LOCALAI_AMD_MOE32_VAR_DOWN", "-1"))
MOE32_SPLITS = int(os.environ.get("LOCALAI_AMD_MOE32_SPLITS", "0"))   # 0: picked from the tile count
MOE32_TILES = {0: (64, 128), 1: (64, 128), 2: (64, 256), 3: (64, 256), 4: (64, 256), 5: (32, 128), 6: (128, 128),
               7: (64, 128), 8: (64, 128), 9: (32, 128), 10: (32, 256), 11: (64, 256), 12: (32, 256),
               13: (64, 128), 14: (32, 256), 15: (128, 256), 16: (128, 128), 17: (64, 256), 18: (128, 128),
               19: (128, 512), 20: (128, 256)}
_MOE32_FMTS = (FMT_Q4_K, FMT_Q6_K, FMT_Q8_0)


def moe32_ok(gu: "MoEWeights", down: "MoEWeights", T: int) -> bool:
    """Can the gate|up / down pair of a layer run on la_moe32 for a T-token batch."""
    return (MOE32 and T >= MOE32_MIN_T and gu.desc is not None and down.desc is not None
            and gu.fmt in _MOE32_FMTS and down.fmt in _MOE32_FMTS and gu.K % 256 == 0 and down.K % 256 == 0
            and gu.N % 32 == 0 and down.K == gu.N // 2)


def moe_glu32(x: torch.Tensor, mw: "MoEWeights", order: torch.Tensor, off: torch.Tensor, topk: int, T: int,
              act: int = ACT_SWIGLU, var: Optional[int] = None) -> torch.Tensor:
    """h = act(x Wg^T) * (x Wu^T) for every routed pair: x [T, K] bf16 -> h [T*topk, F] bf16 in
    the grouping's row order (row off[e] + m is pair order[off[e] + m]); rows of pairs routed to
    no local expert stay unwritten (the down projection never reads them)."""
    F = mw.N // 2
    if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.shape[1] != mw.K:
        raise ValueError("moe_glu32: x must be contiguous bf16 [T, K]")
    h = torch.empty(T * topk, F, dtype=torch.bfloat16, device=x.device)
    a = {ACT_SWIGLU: 0, ACT_GEGLU: 3}[act]
    _check(lib().la_moe32(mw.fmt, 1, mw.desc32().data_ptr(), F, mw.K, mw.E, order.data_ptr(), off.data_ptr(), topk,
                          x.data_ptr(), x.shape[1], T, 1, None, h.data_ptr(), F, 0, a,
                          _moe32_var(MOE32_VAR_GLU, T, mw.fmt) if var is None else var, _stream()), "la_moe32")
    return h


def _moe32_var(env: int, T: int, fmt: int = FMT_Q4_K, down: bool = False) -> int:
    if env >= 0:
        return env
    # live-row-block variants (profiles/r6_moe_live.md, Mixtral-8x7B shapes, cold weights): T = 256
    # var 19 (128-row chunks, 8 waves x 64 columns) glu 244 + down 118 us vs var 15's 280 + 131 on
    # the same box and var 4's 315 + 170 on another; T = 64 / 128
    # var 17 (64-row chunks) 167 + 82 / 172 + 86 vs var 9's 166 + 91 / var 4's 180 + 91; below
    # MOE32_SMALL_T var 9 (32-row tiles, 4 workgroups per CU) stays for the smallest batches
    if T >= MOE32_LIVE_BIG_T:
        # var 19's 64-column waves spill with Q6_K / Q8_0 fragments (the launcher maps them to 15)
        return 19 if fmt == FMT_Q4_K else 15
    return 9 if T < MOE32_SMALL_T else 17


def _moe32_splits(mw: "MoEWeights", T: int, topk: int, var: int) -> int:
    if MOE32_SPLITS:
        S = MOE32_SPLITS
    else:
        bm, bn = MOE32_TILES[var]
        live = (-(-T * topk // bm) + mw.E // 2) * -(-mw.N // bn)   # tiles with rows (balanced router)
        S = 1
        while S < 8 and live * S * 2 <= 1024 and mw.K // 64 >= 64 * S:
            S *= 2
    ks = mw.K // 64
    while S > 1 and -(-ks // S) * (S - 1) >= ks:
        S -= 1
    return S


def moe_down32(h: torch.Tensor, mw: "MoEWeights", order: torch.Tensor, off: torch.Tensor, topk: int, T: int,
               wts: torch.Tensor, zero: bool = False, var: Optional[int] = None) -> Partial:
    """Down projection of moe_glu32's grouped h rows -> Partial [S*topk, T, N]: slab
    (split*topk + slot) row t holds wts[pair] * (h_pair Wd^T) of token t's slot-th pick, so the
    consumer's slab sum is the weighted top-k combine (moe_linear's down contract)."""
    v = _moe32_var(MOE32_VAR_DOWN, T, mw.fmt, down=True) if var is None else var
    S = _moe32_splits(mw, T, topk, v)
    alloc = torch.zeros if zero else torch.empty
    out = alloc(S * topk, T, mw.N, dtype=torch.float32, device=h.device)
    _check(lib().la_moe32(mw.fmt, 2, mw.desc32().data_ptr(), mw.N, mw.K, mw.E, order.data_ptr(), off.data_ptr(), topk,
                          h.data_ptr(), h.shape[1], T, S, wts.data_ptr(), out.data_ptr(), mw.N, T * mw.N, 0, v,
                          _stream()), "la_moe32")
    return Partial(out)


# Grouped MoE on the shared-dequant-image tile (gemm_bs.hip bsmoe_kernel): every local expert's
# routed rows in ONE launch per projection, 256-row tiles (an expert's weights stream once per 256
# rows, not once per 64 as on moe32), grid sized for any routing -- no host read of the grouping.
# Prefill chunks (T >= MOE_BS_MIN_T tokens); decode batches stay on moe32.
# opt-in: slower than both the grouped moe32 tiles and the dense per-expert path on Mixtral-8x7B
# prefill chunks (profiles/r6_moe_live.md)
MOE_BS = os.environ.get("LOCALAI_AMD_MOE_BS", "0") == "1"
MOE_BS_MIN_T = int(os.environ.get("LOCALAI_AMD_MOE_BS_MIN_T", "512"))
MOE_BS_VAR = int(os.environ.get("LOCALAI_AMD_MOE_BS_VAR", "0"))


def moe_bs_ok(gu: "MoEWeights", down: "MoEWeights", T: int) -> bool:
    """Can the gate|up / down pair of a layer run on la_bsmoe for a T-token chunk."""
    return (MOE_BS and T >= MOE_BS_MIN_T and gu.desc is not None and down.desc is not None
            and gu.fmt in _MOE32_FMTS and down.fmt in _MOE32_FMTS and gu.K % 256 == 0 and down.K % 256 == 0
            and gu.N % 16 == 0 and down.N % 4 == 0 and down.K == gu.N // 2)


def moe_glu_bs(x: torch.Tensor, mw: "MoEWeights", order: torch.Tensor, off: torch.Tensor, topk: int, T: int,
               act: int = ACT_SWIGLU, var: Optional[int] = None) -> torch.Tensor:
    """moe_glu32's contract on the bs tile: h [T*topk, F] bf16 in grouped row order."""
    F = mw.N // 2
    if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.shape[1] != mw.K or x.shape[0] != T:
        raise ValueError("moe_glu_bs: x must be contiguous bf16 [T, K]")
    h = torch.empty(T * topk, F, dtype=torch.bfloat16, device=x.device)
    a = {ACT_SWIGLU: 0, ACT_GEGLU: 3}[act]
    _check(lib().la_bsmoe(mw.fmt, 1, mw.desc32().data_ptr(), F, mw.K, mw.E, order.data_ptr(), off.data_ptr(), topk,
                          x.data_ptr(), x.shape[1], T, 1, None, h.data_ptr(), F, 0, a,
                          MOE_BS_VAR if var is None else var, _stream()), "la_bsmoe")
    return h


def moe_down_bs(h: torch.Tensor, mw: "MoEWeights", order: torch.Tensor, off: torch.Tensor, topk: int, T: int,
                wts: torch.Tensor, zero: bool = False, var: Optional[int] = None) -> Partial:
    """moe_down32's contract on the bs tile: Partial [topk, T, N], slab `slot` row t = wts[pair] *
    (h_pair Wd^T) of token t's slot-th pick."""
    if h.dtype != torch.bfloat16 or not h.is_contiguous() or h.shape[1] != mw.K or h.shape[0] != T * topk:
        raise ValueError("moe_down_bs: h must be contiguous bf16 [T*topk, K]")
    alloc = torch.zeros if zero else torch.empty
    out = alloc(topk, T, mw.N, dtype=torch.float32, device=h.device)
    _check(lib().la_bsmoe(mw.fmt, 2, mw.desc32().data_ptr(), mw.N, mw.K, mw.E, order.data_ptr(), off.data_ptr(), topk,
                          h.data_ptr(), h.shape[1], T, 1, wts.data_ptr(), out.data_ptr(), mw.N, T * mw.N, 0,
                          MOE_BS_VAR if var is None else var, _stream()), "la_bsmoe")
    return Partial(out)


MOE_GEMV = os.environ.get("LOCALAI_AMD_MOE_GEMV", "1") == "1"
MOE_GEMV_MAX_T = 2


def moe_gemv_ok(mw: MoEWeights, T: int) -> bool:
    """Decode of 1-2 tokens: the routed experts on the int8-dot GEMV path (gemv_dp4.hip
    moe_gemv_kernel) instead of the MFMA grouped GEMM, which pads each expert's 1-2 rows to 16."""
    return (MOE_GEMV and T <= MOE_GEMV_MAX_T and mw.desc is not None and mw.K % 256 == 0
            and mw.fmt in (FMT_Q4_K, FMT_Q6_K, FMT_Q8_0) and all(w.gemv_ok for w in mw.experts[:1]))


# split-K override of the MoE decode GEMVs (gate|up, down); 0: the dense GEMV's heuristic (A/B knob)
MOE_GEMV_SPLITS = tuple(int(v) for v in os.environ.get("LOCALAI_AMD_MOE_GEMV_SPLITS", "0,0").split(","))


def moe_gemv(x: Optional[torch.Tensor], mw: MoEWeights, ids: torch.Tensor, topk: int, T: int, E_local: int,
             act_src: Optional[Partial] = None, act_mode: int = ACT_SWIGLU,
             wts: Optional[torch.Tensor] = None) -> Partial:
    """gate|up (act_src None): x [T, K] -> Partial [S, T*topk, N] (row = routed pair); down
    (act_src = the gate|up Partial): x = wts[p] * act(gate|up row p) -> Partial [S*topk, T, N],
    the same slab contract as moe_linear.  ids: [T*topk] int32 local expert ids (>= E_local:
    another rank's expert, rows read as zero)."""
    P = T * topk
    S = _gemv_splits([mw.experts[0]], mw.K, 1)
    # one token: its topk routed pairs already multiply the down launch's grid -- half the dense
    # GEMV's splits (Mixtral C=1 8 -> 4: 295.4 -> 300.3 / 294.5 -> 298.5 tok/s; gate|up 2 -> 1
    # neutral; at C=2 quartering both measured 1.3 % slower; r5_mxs*_*.log)
    if T == 1 and act_src is not None:
        nsb = mw.K // 256
        S = max(1, S // 2)
        while nsb % S or (mw.K // S) * (1 + 4 / 16 + 4 / 32) > 65536:
            S += 1
    ov = MOE_GEMV_SPLITS[0 if act_src is None else 1]
    if ov > 0 and (mw.K // 256) % ov == 0 and (mw.K // ov) * (1 + 4 / 16 + 4 / 32) <= 65536:
        S = ov
    dev = ids.device
    if act_src is None:
        out = torch.empty(S, P, mw.N, dtype=torch.float32, device=dev)
        slab = P * mw.N
        _check(lib().la_moe_gemv(mw.fmt, 0, mw.desc.data_ptr(), mw.N, mw.K, E_local, ids.data_ptr(), T, topk,
                                 x.data_ptr(), x.shape[1], S, None, 0, 0, 0, None, out.data_ptr(), mw.N, slab,
                                 _stream()), "la_moe_gemv")
    else:
        a = act_src.src_args()
        if act_src.t.dim() != 3 or a[3]:
            raise ValueError("moe_gemv: the activation source must be fp32 slabs without bias")
        out = torch.empty(S * topk, T, mw.N, dtype=torch.float32, device=dev)
        slab = T * mw.N
        _check(lib().la_moe_gemv(mw.fmt, 1, mw.desc.data_ptr(), mw.N, mw.K, E_local, ids.data_ptr(), T, topk,
                                 None, 0, S, a[0], a[1], a[2], act_mode, wts.data_ptr(), out.data_ptr(), mw.N, slab,
                                 _stream()), "la_moe_gemv")
    return Partial(out)


def grammar_mask(logits: torch.Tensor, slot: torch.Tensor, pool: torch.Tensor) -> None:
    """In-place: logits[b, v] = -inf where pool[slot[b], v] == 0, for rows with slot[b] >= 0
    (grammar-constrained rows whose parse state has a cached allowed-token mask).  pool is
    [slots, >= V] uint8 / bool; slot [B] int32."""
    B, V = logits.shape
    assert pool.shape[1] >= V and slot.shape[0] >= B and slot.dtype == torch.int32
    if not logits.is_cuda:
        for b in range(B):
            s = int(slot[b])
            if s >= 0:
                logits[b].masked_fill_(~pool[s, :V].bool(), float("-inf"))
        return
    if logits.dtype != torch.float32 or logits.stride(1) != 1 or pool.stride(1) != 1:
        raise ValueError("grammar_mask: f32 logits and a row-major pool required")
    _check(lib().la_grammar_mask(logits.data_ptr(), logits.stride(0), B, V, slot.data_ptr(), pool.data_ptr(),
                                 pool.stride(0), _stream()), "la_grammar_mask")


def grammar_advance(tok: torch.Tensor, slot: torch.Tensor, nxt: torch.Tensor) -> None:
    """In-place: for rows with slot >= 0, slot = nxt[slot, tok] if that transition is known
    (>= 0) else -3 (parked: the host drops the row's later tokens of this run).  tok / slot
    int32 [B]; nxt int16 [slots, V]."""
    B = slot.shape[0]
    V = nxt.shape[1]
    assert nxt.dtype == torch.int16 and slot.dtype == torch.int32 and tok.shape[0] >= B
    if not slot.is_cuda:
        for b in range(B):
            s, t = int(slot[b]), int(tok[b])
            if s >= 0:
                ns = int(nxt[s, t]) if 0 <= t < V else -2
                slot[b] = ns if ns >= 0 else -3
        return
    _check(lib().la_grammar_advance(tok.data_ptr(), slot.data_ptr(), nxt.data_ptr(), V, B, _stream()),
           "la_grammar_advance")


def penalties(logits: torch.Tensor, hist: torch.Tensor, hist_len: torch.Tensor, pen: torch.Tensor,
              nl_token: int = -1, penalize_nl: Optional[torch.Tensor] = None, col0: int = 0):
    """In-place repeat/frequency/presence penalties.  hist [B, L] i32 (-1 padded); pen [B,3].
    col0 > 0 or a narrower row: logits hold the vocabulary columns [col0, col0 + V) only (a
    tensor-parallel shard); history tokens outside them are skipped."""
    B = logits.shape[0]
    if not logits.is_cuda:
        V = logits.shape[1]
        for b in range(B):
            L = int(hist_len[b])
            rp, fp, pp = (float(x) for x in pen[b])
            toks = hist[b, :L].tolist()
            for t in set(toks):
                if t < 0:
                    continue
                if t == nl_token and penalize_nl is not None and not bool(penalize_nl[b]):
                    continue
                if t < col0 or t - col0 >= V:
                    continue
                c = toks.count(t)
                v = float(logits[b, t - col0])
                if rp != 1:
                    v = v / rp if v > 0 else v * rp
                v -= c * fp + (pp if c > 0 else 0)
                logits[b, t - col0] = v
        return logits
    _check(lib().la_penalties_cols(logits.data_ptr(), logits.stride(0), B, hist.data_ptr(), hist.stride(0),
                                   hist_len.data_ptr(), pen.data_ptr(), nl_token, _ptr(penalize_nl), col0,
                                   logits.shape[1], _stream()), "la_penalties_cols")
    return logits


# Tensor-parallel sampling over vocabulary shards (sampling.hip tp_* kernels; decoder.TPInfo.sample_cols)
TP_SAMPLE_C = 64   # standard-chain candidates per rank and row: rows with 1 <= top_k <= TP_SAMPLE_C


def tp_topc(logits: torch.Tensor, C: int, base: int, out: torch.Tensor) -> None:
    """out [B, C, 2] f32 (this rank's slot of the exchange buffer): the C largest logits of each row
    of the shard as (value, global id), in increasing id order."""
    B, Vs = logits.shape
    _check(lib().la_tp_topc(logits.data_ptr(), logits.stride(0), B, Vs, C, base, out.data_ptr(), _stream()),
           "la_tp_topc")


def tp_mirostat(phase: int, logits: torch.Tensor, base: int, world: int, rank: int, params_dev: torch.Tensor,
                mu: torch.Tensor, x1: torch.Tensor, x2: torch.Tensor, x3: torch.Tensor, own: Optional[torch.Tensor],
                out_tok: Optional[torch.Tensor]) -> None:
    B, Vs = logits.shape
    _check(lib().la_tp_mirostat(phase, logits.data_ptr(), logits.stride(0), B, Vs, base, world, rank,
                                params_dev.data_ptr(), mu.data_ptr(), x1.data_ptr(), x2.data_ptr(), x3.data_ptr(),
                                _ptr(own), _ptr(out_tok), _stream()), "la_tp_mirostat")


def penalty_push(nxt: torch.Tensor, hist: torch.Tensor, cnt: torch.Tensor, hl: torch.Tensor,
                 cap: torch.Tensor) -> None:
    """Append the sampled tokens to each row's penalty ring (hist [B, L] i32, ring size cap[b])
    and refresh hist_len = min(count, cap) -- the in-graph history the penalties kernel reads."""
    B = nxt.shape[0]
    if not nxt.is_cuda:
        for b in range(B):
            k = int(cap[b])
            if k <= 0:
                continue
            c = int(cnt[b])
            hist[b, c % k] = nxt[b]
            cnt[b] = c + 1
            hl[b] = min(c + 1, k)
        return
    _check(lib().la_pen_push(nxt.data_ptr(), B, hist.data_ptr(), hist.stride(0), cnt.data_ptr(), hl.data_ptr(),
                             cap.data_ptr(), _stream()), "la_pen_push")


# ---------------------------------------------------------------------------------------
# Mamba decode step (mamba.hip)
# ---------------------------------------------------------------------------------------

def mamba_conv_step(conv_state: torch.Tensor, xz: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
                    out: torch.Tensor) -> torch.Tensor:
    """conv_state [B, I, K] fp32 (rolled in place); xz [B, >=2I] fp32; w [I, K] fp32 -> out [B, I]."""
    B, I, K = conv_state.shape
    for t in (conv_state, xz, w, out):
        assert t.dtype == torch.float32 and t.is_cuda and t.stride(-1) == 1
    assert conv_state.is_contiguous() and w.shape == (I, K) and out.shape == (B, I) and out.is_contiguous()
    assert xz.shape[0] == B and xz.shape[1] >= 2 * I and (bias is None or bias.shape == (I,))
    _check(lib().la_mamba_conv_step(conv_state.data_ptr(), xz.data_ptr(), xz.stride(0), w.data_ptr(),
                                    None if bias is None else bias.data_ptr(), out.data_ptr(), B, I, K, _stream()),
           "la_mamba_conv_step")
    return out


def mamba_ssm_step(ssm_state: torch.Tensor, x: torch.Tensor, dt: torch.Tensor, bc: torch.Tensor, off_b: int,
                   off_c: int, A: torch.Tensor, D: torch.Tensor, xz: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """Selective-state update of one token: ssm_state [B, I, N] fp32 (in place), x / dt [B, I],
    bc [B, *] holding B at off_b and C at off_c, A [I, N] (negative), D [I], z = xz[:, I:2I]."""
    B, I, N = ssm_state.shape
    for t in (ssm_state, x, dt, bc, A, D, xz, out):
        assert t.dtype == torch.float32 and t.is_cuda and t.stride(-1) == 1
    assert ssm_state.is_contiguous() and x.is_contiguous() and dt.is_contiguous() and out.is_contiguous()
    assert A.shape == (I, N) and D.shape == (I,) and bc.shape[0] == B and bc.shape[1] >= max(off_b, off_c) + N
    assert xz.shape[0] == B and xz.shape[1] >= 2 * I
    _check(lib().la_mamba_ssm_step(ssm_state.data_ptr(), x.data_ptr(), dt.data_ptr(), bc.data_ptr(), bc.stride(0),
                                   off_b, off_c, A.data_ptr(), D.data_ptr(), xz.data_ptr(), xz.stride(0),
                                   out.data_ptr(), B, I, N, _stream()), "la_mamba_ssm_step")
    return out


# ---------------------------------------------------------------------------------------
# GroupNorm (+ SiLU) over NHWC bf16 activations (groupnorm.hip) -- the SD UNet / VAE norms
# ---------------------------------------------------------------------------------------

def groupnorm_supported(x: torch.Tensor, groups: int) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    C = x.shape[1]
    return (x.is_contiguous(memory_format=torch.channels_last) and groups <= 64 and 256 % (2 * groups) == 0
            and C % groups == 0
            and (C // groups) % 2 == 0 and C <= 2048)


# ---------------------------------------------------------------------------------------
# Image preprocessing (K26): PIL-exact bicubic resample + placement + normalise + tiles
# ---------------------------------------------------------------------------------------

def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


@functools.lru_cache(maxsize=64)
def pil_bicubic_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """PIL's precompute_coeffs + normalize_coeffs_8bpc for BICUBIC (Resample.c): per output
    index the first source index and count, and int32 weights in 22-bit fixed point."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        for x in range(xmax):
            c = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + c * (1 << 22)) if c < 0 else int(0.5 + c * (1 << 22))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


_IMG_TABLES: dict = {}


def _img_tables(in_size: int, out_size: int, device):
    key = (in_size, out_size, str(device))
    t = _IMG_TABLES.get(key)
    if t is None:
        b, k, ks = pil_bicubic_coeffs(in_size, out_size)
        t = _IMG_TABLES[key] = (torch.from_numpy(b).to(device), torch.from_numpy(k).to(device), ks)
    return t


def image_tiles(img: torch.Tensor, placements: Sequence[dict], out: torch.Tensor, mean, std) -> torch.Tensor:
    """img: uint8 [H, W, 3] on the GPU.  Each placement resizes the image to (ow, oh) with PIL's
    BICUBIC (bit-exact), puts it at (ox, oy) on a (cw, ch) canvas filled with `fill`, and writes the
    canvas' S x S tiles, normalised, into out[t0 + i] (out: fp32 [n, 3, S, S])."""
    H, W, _ = img.shape
    S = out.shape[-1]
    assert img.dtype == torch.uint8 and img.is_contiguous() and out.is_contiguous() and out.dtype == torch.float32
    m = torch.tensor(list(mean), dtype=torch.float32, device=img.device)
    sd = torch.tensor(list(std), dtype=torch.float32, device=img.device)
    for pl in placements:
        ow, oh, cw, ch = int(pl["ow"]), int(pl["oh"]), int(pl["cw"]), int(pl["ch"])
        if cw % S or ch % S or pl["t0"] + (cw // S) * (ch // S) > out.shape[0]:
            raise ValueError("image_tiles: canvas does not tile the output")
        bh, kh, ksh = _img_tables(W, ow, img.device)
        bv, kv, ksv = _img_tables(H, oh, img.device)
        tmp = torch.empty(H, ow, 3, dtype=torch.uint8, device=img.device)
        _check(lib().la_img_resample_h(img.data_ptr(), H, W, tmp.data_ptr(), ow, bh.data_ptr(), kh.data_ptr(), ksh,
                                       _stream()), "la_img_resample_h")
        fill = torch.tensor(list(pl.get("fill", (0, 0, 0))), dtype=torch.int32, device=img.device)
        _check(lib().la_img_resample_v_tiles(tmp.data_ptr(), oh, ow, bv.data_ptr(), kv.data_ptr(), ksv, ch, cw,
                                             int(pl.get("oy", 0)), int(pl.get("ox", 0)), S, int(pl["t0"]),
                                             m.data_ptr(), sd.data_ptr(), fill.data_ptr(), out.data_ptr(), _stream()),
               "la_img_resample_v_tiles")
    return out


def groupnorm_nhwc(x: torch.Tensor, groups: int, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
                   eps: float, silu: bool = False) -> torch.Tensor:
    """x [B, C, H, W] bf16 in channels_last memory -> GroupNorm(x) (SiLU'd when `silu`), same layout."""
    assert groupnorm_supported(x, groups), "groupnorm_nhwc: bf16 channels_last, even channels per group, C <= 2048"
    B, C, H, W = x.shape
    for t in (weight, bias):
        assert t is None or (t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() == C)
    HW = H * W
    rows_s = max(1, -(-HW * B // 256))    # statistics: ~256 workgroups, few partials
    rows_a = max(1, -(-HW * B // 1024))   # apply: ~1024 workgroups over the chip
    S = -(-HW // rows_s)
    part = torch.empty(B * S * groups * 2, dtype=torch.float32, device=x.device)
    y = torch.empty_like(x, memory_format=torch.channels_last)
    _check(lib().la_groupnorm_nhwc(x.data_ptr(), y.data_ptr(), _ptr(weight), _ptr(bias), part.data_ptr(), B, HW, C,
                                   groups, rows_s, rows_a, float(eps), int(silu), _stream()), "la_groupnorm_nhwc")
    return y
