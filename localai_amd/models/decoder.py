"""Decoder-only transformer families served by the engine: llama (Llama-2/3, Mistral, Yi,
DeepSeek-coder), llama+MoE (Mixtral), phi2, phi3, qwen2, gemma, gemma2, command-r, starcoder2.

Replaces the llama.cpp graph the reference's backend drives through llama_decode
(`backend/cpp/llama/grpc-server.cpp:1910`, [external]).  The forward pass is a fixed
sequence of our gfx950 kernels (ops/csrc):

  embed(K1) -> [ add_norm(K2+K14) -> QKV skinny/hipBLASLt GEMM (K5/K6) -> rope_kv (K9+K10)
             -> paged attention (K12) -> O GEMM -> add_norm -> gate|up GEMM -> act (K13)
             -> down GEMM ] x L -> add_norm -> lm_head GEMM -> on-device sampler (K22)

Tensor parallelism (one process per GPU, RCCL over xGMI via torch.distributed "nccl"):
column-parallel QKV / gate|up (heads and FFN columns split), row-parallel O / down
(K split along 256-aligned super-blocks), one all-reduce after each row-parallel GEMM,
vocab-parallel lm_head + all-gather.  Experts (Mixtral) are split the same way
(TP-within-expert).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..gguf import GGML_BLOCK, GGMLType, GGUFReader, dequantize, quantize
from .hparams import HParams

# batch-1/2 decode: q|k|v GEMV with RoPE + KV append in its epilogue (ops.qkv_rope_dp4)
FUSED_QKV_ROPE = os.environ.get("LOCALAI_AMD_QKV_ROPE", "1") == "1"
# tensor parallelism: row-parallel outputs of at least this many rows (prefill chunks) all-reduce
# chunk by chunk on a comm stream, overlapped with the next chunk's GEMM
TP_OVERLAP_ROWS = int(os.environ.get("LOCALAI_AMD_TP_OVERLAP_ROWS", "1024"))
TP_OVERLAP_CHUNKS = int(os.environ.get("LOCALAI_AMD_TP_OVERLAP_CHUNKS", "4"))
# MoE decode batches route with the fused router kernel (moe.hip); =1 falls back to the torch ops
FUSED_ROUTER_OFF = os.environ.get("LOCALAI_AMD_FUSED_ROUTER_OFF", "0") == "1"
# prefill chunks of at least this many tokens run each expert as a dense GEMM over its gathered
# rows (~T * topk / E rows: weights dequantised once per expert + the library GEMM, one host read
# of the grouping).  Below it every batch runs the grouped moe32 tiles (no host sync).  Measured
# on Mixtral-8x7B shapes (profiles/r6_moe_live.md): T = 8192 dense 6.36 ms vs grouped moe32 7.42 /
# bs 7.65; T = 4096 grouped moe32 3.53 ms vs dense 4.06; T = 1024 1.07 vs 1.85; HTTP C=256
# 10.61 k tok/s / p50 TTFT 1128 ms with dense 8192-token chunks vs 10.14 k / 1245 ms on the
# grouped bs tile
MOE_DENSE_MIN_T = int(os.environ.get("LOCALAI_AMD_MOE_DENSE_MIN_T", "6144"))

_ACT = {"swiglu": ops.ACT_SWIGLU, "gelu": ops.ACT_GELU, "geglu": ops.ACT_GEGLU}


TP_AR_BF16 = os.environ.get("LOCALAI_AMD_TP_AR_BF16", "1") == "1"
TP_AR_BF16_MAX_ROWS = 512           # decode batches only; prefill chunks reduce in fp32
ALLREDUCE_ADD_NORM_MAX_SLABS = 64   # allreduce.hip la_allreduce_add_norm rejects more split-K slabs


class CustomAllReduceTimeout(RuntimeError):
    pass


@dataclass
class PendingAR:
    """A row-parallel output whose all-reduce is deferred to its consumer, the layer-boundary
    add_norm: CustomAllReduce.add_norm then runs slab sum + all-reduce + bias + residual + norm as
    ONE launch (decode steps of a GPU TP group).  Deliberately not an ops.Partial: any other
    consumer fails loudly instead of reading a rank-local partial sum."""
    part: "ops.Partial"
    bias: Optional[torch.Tensor]


@dataclass
class TPInfo:
    rank: int = 0
    world: int = 1
    group: object = None
    car: object = None  # parallel.custom_ar.CustomAllReduce (one-shot over xGMI peer buffers) or None
    ep: bool = False    # MoE layers: expert parallelism (each rank holds E/world whole experts)

    def all_reduce(self, t: torch.Tensor):
        if self.world > 1:
            if self.car is not None and self.car.supports(t):
                return self.car.all_reduce(t)   # latency-bound decode rows
            import torch.distributed as dist
            dist.all_reduce(t, group=self.group)  # RCCL: prefill chunks, CPU (gloo)
        return t

    def drop_custom_ar(self) -> None:
        car, self.car = self.car, None
        if car is not None:
            car.close()

    def check_custom_ar(self, ctrl) -> None:
        """Called once per engine step, at a host sync point that exists anyway: if ANY rank's
        one-shot all-reduce hit its spin limit (a peer arrived too late: that call summed stale or
        partial peer slots), every rank agrees over the gloo control group to drop the custom
        path -- RCCL from then on -- and the step fails loudly instead of serving wrong sums."""
        if self.world < 2 or self.car is None:
            return
        import torch.distributed as dist
        bad = torch.tensor([1 if self.car.timed_out() else 0], dtype=torch.int32)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=ctrl)
        if int(bad.item()):
            car, self.car = self.car, None
            car.close()
            raise CustomAllReduceTimeout("tensor-parallel one-shot all-reduce timed out on a late peer rank: this "
                                         "step's results are invalid; the group continues on RCCL")

    def comm_stream(self, device) -> "torch.cuda.Stream":
        """The TP collectives' own HIP stream (prefill all-reduces overlapped with GEMMs)."""
        st = getattr(self, "_comm", None)
        if st is None:
            st = self._comm = torch.cuda.Stream(device=device)
        return st

    def argmax_cols(self, t: torch.Tensor) -> torch.Tensor:
        """Greedy token (int32 [B]) of every row of vocab-parallel logits t [B, V / world] (this
        rank's columns): local max and argmax, then ONE exchange of the B x 2 candidates and the
        max over ranks (first maximum: the lowest id on ties, as the shards are in rank order).
        Exact, and with the custom all-reduce present graph-capturable with no RCCL call: the
        candidates ride a zero-padded one-shot all-reduce (0 + v sums exactly in fp32).  The
        decode graph thereby moves B x world x 8 bytes instead of the B x V fp32 all-gather."""
        B, Vs = t.shape
        v, i = t.float().max(-1)
        if self.world == 1:
            return i.to(torch.int32)
        if Vs * self.world >= (1 << 24):
            raise ValueError("argmax_cols: token ids must be exact in fp32")
        gid = (i + self.rank * Vs).float()
        buf = torch.zeros(self.world, B, 2, dtype=torch.float32, device=t.device)
        if self.car is not None and self.car.supports(buf):
            buf[self.rank, :, 0] = v
            buf[self.rank, :, 1] = gid
            self.car.all_reduce(buf.view(-1))
        else:
            import torch.distributed as dist
            parts = list(buf.unbind(0))
            dist.all_gather(parts, torch.stack([v, gid], -1), group=self.group)
            buf = torch.stack(parts, 0)
        best = buf[..., 0].argmax(0, keepdim=True)                       # [1, B]: first max -> lowest rank
        return buf[..., 1].gather(0, best).squeeze(0).to(torch.int32)

    def sample_workspace(self, B: int, device) -> dict:
        """Exchange buffers of sample_cols for batches of B rows (allocated once per captured graph:
        a replayed graph keeps using the same memory)."""
        C, w = ops.TP_SAMPLE_C, self.world
        f32 = dict(dtype=torch.float32, device=device)
        return {"cand": torch.zeros(w, B, C, 2, **f32), "x1": torch.zeros(w, B, 3, **f32),
                "x2": torch.zeros(w, B, **f32), "x3": torch.zeros(w, B, 2, **f32), "mu_tmp": torch.zeros(B, **f32),
                "idx": torch.zeros(B, dtype=torch.int32, device=device)}

    def _exchange(self, buf: torch.Tensor) -> None:
        """Sum `buf` over the group, in place: every rank filled only its own slot, so the sum is
        the concatenation of all slots.  The custom all-reduce when it takes the size (graph-
        replayable, no RCCL call in a captured step), else the process group."""
        if self.car is not None and self.car.supports(buf.view(-1)):
            self.car.all_reduce(buf.view(-1))
        else:
            import torch.distributed as dist
            dist.all_reduce(buf, group=self.group)

    def sample_cols(self, t: torch.Tensor, prm_np, prm_dev: torch.Tensor, mu: torch.Tensor, out: torch.Tensor,
                    ws: dict, mirostat: bool = True) -> torch.Tensor:
        """The device sampler over vocabulary-parallel logits t [B, V / world] (this rank's columns,
        bias and penalties applied), without gathering a row (ref: vLLM's TP sampling behind
        backend/python/vllm/backend.py:102-103; SURVEY §2.9 distributed top-k):
          * greedy and standard-chain rows (1 <= top_k <= TP_SAMPLE_C): every rank's top-C
            candidates (value, id) -- together a superset of the global top-k, which is all the
            chain after top-k looks at -- are exchanged in ONE sum all-reduce of [world, B, C, 2]
            and the unchanged sampler kernel runs on the merged [B, world * C] rows (in global id
            order, so its lowest-id tie breaks are the full row's); Philox stream as at TP=1;
          * mirostat-2 rows: four phases with three [world, B, <=3] exchanges (local max / argmax /
            sum-exp, kept mass per rank, the pick of the rank holding the draw), the mu update
            computed alike on every rank.
        Graph-capturable with the custom all-reduce (no RCCL call).  out: int32 [B] tokens."""
        B, Vs = t.shape
        base, w, C = self.rank * Vs, self.world, ops.TP_SAMPLE_C
        cand = ws["cand"]
        cand.zero_()
        ops.tp_topc(t, C, base, cand[self.rank])
        self._exchange(cand)
        vals = cand[..., 0].permute(1, 0, 2).contiguous().view(B, w * C)   # unit column stride for the sampler
        ids = cand[..., 1].permute(1, 0, 2).contiguous().view(B, w * C)
        ops.sample(vals, prm_np, mu=ws["mu_tmp"], params_dev=prm_dev, out=ws["idx"])
        out.copy_(ids.gather(1, ws["idx"].long().unsqueeze(1)).squeeze(1).to(torch.int32))
        if mirostat:
            x1, x2, x3 = ws["x1"], ws["x2"], ws["x3"]
            x1.zero_()
            x2.zero_()
            x3.zero_()
            ops.tp_mirostat(1, t, base, w, self.rank, prm_dev, mu, x1, x2, x3, x1[self.rank], None)
            self._exchange(x1)
            ops.tp_mirostat(2, t, base, w, self.rank, prm_dev, mu, x1, x2, x3, x2[self.rank], None)
            self._exchange(x2)
            ops.tp_mirostat(3, t, base, w, self.rank, prm_dev, mu, x1, x2, x3, x3[self.rank], None)
            self._exchange(x3)
            ops.tp_mirostat(4, t, base, w, self.rank, prm_dev, mu, x1, x2, x3, None, out)
        return out

    def all_gather_cols(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        import torch.distributed as dist
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, -1)


@dataclass
class ForwardBatch:
    tokens: torch.Tensor                 # [T] i32
    pos: torch.Tensor                    # [T] i32
    slots: torch.Tensor                  # [T] i32  (-1: no KV write)
    decode: bool
    block_tables: torch.Tensor           # [nseq, maxb] i32
    seq_lens: Optional[torch.Tensor] = None   # decode: [B] i32 (keys incl. the new one)
    max_len: int = 0                          # decode: upper bound of seq_lens
    cu_q: Optional[torch.Tensor] = None       # prefill: [nseq+1] i32
    ctx_lens: Optional[torch.Tensor] = None   # prefill: [nseq] i32
    tiles: Optional[torch.Tensor] = None      # prefill: attention work tiles
    logits_idx: Optional[torch.Tensor] = None  # rows to project to logits (None: all)
    inject_idx: Optional[torch.Tensor] = None  # prefill rows whose embedding is given (images)
    inject_rows: Optional[torch.Tensor] = None  # [n, n_embd] f32


class KVCache:
    """Per-layer paged K/V pools: K [num_blocks, Hkv_local, block_size, head_dim], V transposed in
    groups of 8 keys [num_blocks, Hkv_local, block_size/8, head_dim, 8] (bf16)."""

    def __init__(self, n_layer: int, num_blocks: int, n_kv: int, block_size: int, head_dim: int, device,
                 dtype=torch.bfloat16):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.k = [torch.zeros(num_blocks, n_kv, block_size, head_dim, dtype=dtype, device=device)
                  for _ in range(n_layer)]
        # V pages are stored transposed per 8-key group ([block_size/8][head_dim][8]) -- see
        # ops/csrc/attention.hip
        if block_size % 8:
            raise ValueError(f"block_size {block_size} must be a multiple of 8")
        self.v = [torch.zeros(num_blocks, n_kv, block_size // 8, head_dim, 8, dtype=dtype, device=device)
                  for _ in range(n_layer)]

    @staticmethod
    def bytes_per_block(n_layer, n_kv, block_size, head_dim, dtype_bytes=2):
        return 2 * n_layer * n_kv * block_size * head_dim * dtype_bytes


@dataclass
class Layer:
    attn_norm: torch.Tensor
    attn_norm_b: Optional[torch.Tensor]
    qkv: List[ops.QWeight]
    qkv_bias: Optional[torch.Tensor]
    wo: ops.QWeight
    wo_bias: Optional[torch.Tensor]
    ffn_norm: Optional[torch.Tensor]
    ffn_norm_b: Optional[torch.Tensor]
    gate_up: List[ops.QWeight]
    up_bias: Optional[torch.Tensor]
    down: Optional[ops.QWeight]
    down_bias: Optional[torch.Tensor]
    router: Optional[torch.Tensor] = None            # [E, D] f32 (MoE)
    experts: Optional[List[tuple]] = None            # [(gate_up list, down)] per expert
    moe_gu: Optional[object] = None                  # ops.MoEWeights (fused gate|up of every expert)
    moe_down: Optional[object] = None                # ops.MoEWeights
    post_attn_norm: Optional[torch.Tensor] = None    # Gemma-2: RMSNorm of the attention output
    post_ffw_norm: Optional[torch.Tensor] = None     # Gemma-2: RMSNorm of the MLP output
    window: int = 0                                  # sliding-window attention span (0: full)
    shexp_gate_up: Optional[List[ops.QWeight]] = None  # Qwen2-MoE shared expert (TP-sliced like a dense MLP)
    shexp_down: Optional[ops.QWeight] = None
    shexp_gate: Optional[torch.Tensor] = None        # [D] f32: sigmoid(x . g) scales the shared expert
    mla: Optional[dict] = None                       # DeepSeek-V2 latent attention weights (see _mla_qkv)
    F: int = 0                                       # this layer's FFN width when it differs from self.F


def _raw2d(t, rows: Optional[slice] = None, cols: Optional[slice] = None):
    """Slice a GGUF tensor's raw bytes as a 2-D [N, K] matrix by rows and/or column blocks.
    A column shard that does not fall on quant-block boundaries (small models at high TP
    degree) is dequantised and returned as BF16."""
    N, K = t.shape[-2], t.shape[-1]
    bs, bb = GGML_BLOCK[t.ggml_type]
    if cols is not None and (cols.start % bs or cols.stop % bs):
        w = dequantize(t.data, t.ggml_type, (N, K))
        if rows is not None:
            w = w[rows]
        w = np.ascontiguousarray(w[:, cols])
        return quantize(w, GGMLType.BF16), w.shape, GGMLType.BF16
    a = t.data.reshape(-1, K // bs, bb)
    if rows is not None:
        a = a[rows]
    n = a.shape[0]
    k = K
    if cols is not None:
        b0, b1 = cols.start // bs, cols.stop // bs
        a = a[:, b0:b1]
        k = cols.stop - cols.start
    return np.ascontiguousarray(a).reshape(-1), (n, k), t.ggml_type


class DecoderModel:
    _defer_ar = False  # set per forward: decode all-reduces fused into the next add_norm (PendingAR)

    def __init__(self, reader: GGUFReader, device: torch.device, tp: Optional[TPInfo] = None,
                 max_pos: Optional[int] = None, rope_overrides: Optional[dict] = None, lora=None):
        self.hp = hp = HParams.from_gguf(reader)
        self.device = device
        self.tp = tp = tp or TPInfo()
        W, R = tp.world, tp.rank
        # more ranks than kv heads (Qwen2-7B's 4 kv heads at TP=8, Gemma-2B's 1): each kv head is
        # replicated on the W / n_head_kv ranks whose query heads read it (their GQA groups line up)
        self.kv_rep = W // hp.n_head_kv if W > hp.n_head_kv and W % hp.n_head_kv == 0 else 1
        if hp.n_head % W or (hp.n_head_kv % W and self.kv_rep == 1):
            raise ValueError(f"TP={W} must divide the query heads ({hp.n_head}) and divide or be a multiple of "
                             f"the kv heads ({hp.n_head_kv})")
        self.Hq, self.Hkv, self.Dh = hp.n_head // W, max(1, hp.n_head_kv // W), hp.head_dim
        if hp.kv_lora_rank:
            if W > 1:
                raise ValueError("DeepSeek-V2 latent attention runs on a single GPU (no tensor parallelism)")
            # MLA decompresses K and V per query head: the cache holds n_head heads of the key
            # width (V padded to it, see _mla_qkv)
            self.Hkv = hp.n_head
        self.F = hp.n_ff // W
        # expert parallelism: rank R holds experts [R*El, (R+1)*El) whole (no F split).  The MoE input
        # is replicated across the group (it follows the attention all-reduce), so each rank runs its
        # local experts for the tokens routed to them and the same all-reduce that closes a TP MLP
        # sums the experts' weighted outputs: no all-to-all is needed with replicated activations.
        self.ep = bool(tp.ep and hp.n_expert and W > 1)
        if self.ep and hp.n_expert % W:
            raise ValueError(f"expert parallelism {W} must divide the expert count {hp.n_expert}")
        self.E_local = hp.n_expert // W if self.ep else hp.n_expert
        self.ep_base = R * self.E_local if self.ep else 0
        if self.ep:
            self.F = hp.n_ff
        self.rot = hp.rope_dim or hp.head_dim
        self.scale = hp.attn_scale or 1.0 / math.sqrt(hp.head_dim)
        self.norm_mode = 0 if hp.norm_type == "rms" else 1
        T = reader.tensors
        dev = device
        def f32(name):
            if name not in T:
                return None
            t = T[name]
            arr = dequantize(t.data, t.ggml_type, t.shape).reshape(-1).astype(np.float32)
            return torch.from_numpy(arr).to(dev)

        def qw(name, rows=None, cols=None):
            if lora is not None and name in lora:
                # LoRA-adapted weight: base + deltas merged in fp32, kept as BF16 (models/lora.py)
                t = T[name]
                w = lora.merged(name, dequantize(t.data, t.ggml_type, t.shape).reshape(t.shape[-2], t.shape[-1]))
                if rows is not None:
                    w = w[rows]
                if cols is not None:
                    w = w[:, cols]
                w = np.ascontiguousarray(w)
                return ops.QWeight.from_raw(quantize(w, GGMLType.BF16), GGMLType.BF16, w.shape, dev)
            raw, shape, gt = _raw2d(T[name], rows, cols)
            return ops.QWeight.from_raw(raw, gt, shape, dev)

        def sl(n_total, part=None):
            n = n_total // W
            return slice(R * n, (R + 1) * n)

        def vec_slice(v, s):
            return None if v is None else v[s].contiguous()

        qd, kvd = hp.q_dim, hp.kv_dim
        self.tok_embd = qw("token_embd.weight")
        self.layers: List[Layer] = []
        for i in range(hp.n_layer):
            b = f"blk.{i}."
            qs, ks = sl(qd), sl(kvd)
            mla = None
            if hp.kv_lora_rank:
                mla = self._load_mla(b, T, qw, f32)
            if self.kv_rep > 1:  # this rank's (replicated) kv head
                kvh = R // self.kv_rep
                ks = slice(kvh * hp.head_dim, (kvh + 1) * hp.head_dim)
            if mla is not None:
                qkv, qkv_bias = [], None
            elif b + "attn_qkv.weight" in T:  # phi-2 / phi-3: one fused [q; k; v] projection
                qkv_name = b + "attn_qkv.weight"
                qkv = [qw(qkv_name, rows=slice(qs.start, qs.stop)),
                       qw(qkv_name, rows=slice(qd + ks.start, qd + ks.stop)),
                       qw(qkv_name, rows=slice(qd + kvd + ks.start, qd + kvd + ks.stop))]
                qb = f32(b + "attn_qkv.bias")
                qkv_bias = None if qb is None else torch.cat([qb[qs], qb[qd + ks.start:qd + ks.stop],
                                                              qb[qd + kvd + ks.start:qd + kvd + ks.stop]])
            else:
                qkv = [qw(b + "attn_q.weight", rows=qs), qw(b + "attn_k.weight", rows=ks),
                       qw(b + "attn_v.weight", rows=ks)]
                qkv_bias = None
                if b + "attn_q.bias" in T:
                    qkv_bias = torch.cat([f32(b + "attn_q.bias")[qs], f32(b + "attn_k.bias")[ks],
                                          f32(b + "attn_v.bias")[ks]])
            qkv = ops.fuse_runs(qkv) if qkv else qkv  # q|k|v, or q|k + v when v has its own format (Q4_K_M)
            wo = qw(b + "attn_output.weight", cols=sl(hp.n_head * hp.head_dim_v if mla is not None else qd))
            wo_b = f32(b + "attn_output.bias")
            if wo_b is not None and R != 0:
                wo_b = torch.zeros_like(wo_b)  # bias added once across TP ranks
            fs = sl(hp.n_ff)
            ff_exp = hp.n_ff_exp or hp.n_ff  # expert width (DeepSeek-V2: != the dense layers' n_ff)
            router = experts = None
            gate_up, down, up_b, down_b = [], None, None, None
            moe_layer = hp.n_expert and i >= hp.n_layer_dense_lead and b + "ffn_gate_inp.weight" in T
            if moe_layer and b + "exp_probs_b.bias" in T:
                raise ValueError(f"{b}exp_probs_b: expert-selection bias (DeepSeek-V3 routing) is not supported")
            if moe_layer:
                router = f32(b + "ffn_gate_inp.weight").view(hp.n_expert, hp.n_embd)
                experts = []
                for e in range(self.ep_base, self.ep_base + self.E_local):
                    efs = None if self.ep else sl(ff_exp)  # EP: whole experts, TP-within-expert: F slices
                    ge = self._expert_slice(T[b + "ffn_gate_exps.weight"], e, rows=efs)
                    ue = self._expert_slice(T[b + "ffn_up_exps.weight"], e, rows=efs)
                    de = self._expert_slice(T[b + "ffn_down_exps.weight"], e, cols=None if self.ep else sl(ff_exp))
                    gu = ops.concat_rows([ge, ue])
                    experts.append(([gu] if gu is not None else [ge, ue], de))
            elif b + "ffn_gate.weight" not in T and hp.act == "gelu":  # phi-2 / starcoder2: up -> gelu -> down
                gate_up = [qw(b + "ffn_up.weight", rows=fs)]
                up_b = vec_slice(f32(b + "ffn_up.bias"), fs)
                down = qw(b + "ffn_down.weight", cols=fs)
                down_b = f32(b + "ffn_down.bias")
                if down_b is not None and R != 0:
                    down_b = torch.zeros_like(down_b)
            else:
                if b + "ffn_gate.weight" in T:
                    g, u = qw(b + "ffn_gate.weight", rows=fs), qw(b + "ffn_up.weight", rows=fs)
                else:  # phi-3: ffn_up holds [gate; up] (2 n_ff rows)
                    g = qw(b + "ffn_up.weight", rows=fs)
                    u = qw(b + "ffn_up.weight", rows=slice(hp.n_ff + fs.start, hp.n_ff + fs.stop))
                gu = ops.concat_rows([g, u])
                gate_up = [gu] if gu is not None else [g, u]
                down = qw(b + "ffn_down.weight", cols=fs)
            shexp_gu = shexp_down = shexp_gate = None
            if b + "ffn_up_shexp.weight" in T:
                fsh = sl(hp.n_ff_shexp)  # sliced by rank even under EP: the all-reduce sums it once
                g, u = qw(b + "ffn_gate_shexp.weight", rows=fsh), qw(b + "ffn_up_shexp.weight", rows=fsh)
                gu = ops.concat_rows([g, u])
                shexp_gu = [gu] if gu is not None else [g, u]
                shexp_down = qw(b + "ffn_down_shexp.weight", cols=fsh)
                shexp_gate = f32(b + "ffn_gate_inp_shexp.weight")
            moe_gu = moe_down = None
            if experts and all(len(gu) == 1 for gu, _ in experts):
                try:
                    moe_gu = ops.MoEWeights([gu[0] for gu, _ in experts])
                    moe_down = ops.MoEWeights([d for _, d in experts])
                except ValueError:
                    moe_gu = moe_down = None
            self.layers.append(Layer(
                attn_norm=f32(b + "attn_norm.weight"), attn_norm_b=f32(b + "attn_norm.bias"),
                qkv=qkv, qkv_bias=qkv_bias, wo=wo, wo_bias=wo_b,
                ffn_norm=f32(b + "ffn_norm.weight"), ffn_norm_b=f32(b + "ffn_norm.bias"),
                gate_up=gate_up, up_bias=up_b, down=down, down_bias=down_b,
                router=router, experts=experts, moe_gu=moe_gu, moe_down=moe_down,
                shexp_gate_up=shexp_gu, shexp_down=shexp_down, shexp_gate=shexp_gate, mla=mla,
                F=(ff_exp if moe_layer else hp.n_ff) // W if hp.n_ff_exp else 0,
                post_attn_norm=f32(b + "post_attention_norm.weight"), post_ffw_norm=f32(b + "post_ffw_norm.weight"),
                # Gemma-2 alternates sliding-window (even) and global (odd) layers
                window=hp.sliding_window if hp.sliding_window and i % 2 == 0 else 0))
        self.out_norm = f32("output_norm.weight")
        self.out_norm_b = f32("output_norm.bias")
        vs = sl(hp.n_vocab)
        self.vocab_local = vs.stop - vs.start
        if hp.n_vocab % W:
            raise ValueError("TP must divide the vocabulary")
        out_name = "output.weight" if "output.weight" in T else "token_embd.weight"
        self.output = qw(out_name, rows=vs)
        ob = f32("output.bias")
        self.out_bias = None if ob is None else ob[vs].contiguous()
        rope_freqs = f32("rope_freqs.weight")
        self.max_pos = max_pos or hp.n_ctx_train
        ro = rope_overrides or {}
        theta = ro.get("freq_base") or hp.rope_theta
        fscale = ro.get("freq_scale") or hp.rope_freq_scale
        yarn = ro.get("yarn")
        if yarn is None and ro.get("type", hp.rope_scaling) == "yarn":
            # YaRN declared in the GGUF (rope.scaling.*): DeepSeek-V2 passes the rotation an
            # attn_factor of 1 / (1 + 0.1 ln(1 / freq_scale)) so cos/sin stay unscaled and the
            # magnitude correction lives in the query scale (HParams.attn_scale)
            yarn = {"orig_ctx": hp.rope_orig_ctx or hp.n_ctx_train,
                    "attn_factor": 1.0 / (1.0 + 0.1 * math.log(1.0 / fscale))
                    if hp.kv_lora_rank and fscale < 1.0 else 1.0}
        self.cos_sin = ops.rope_cos_sin(self.max_pos, self.rot, theta, dev, freq_scale=fscale,
                                        freq_factors=rope_freqs, rope_type=ro.get("type", hp.rope_scaling),
                                        yarn=yarn)

    def _load_mla(self, b: str, T, qw, f32) -> dict:
        """DeepSeek-V2 latent-attention weights (llama.cpp build_deepseek2 [external]).  The q
        projection's rows are reordered per head from [nope | rope] to [rope | nope] so the rotary
        part is the head's FIRST n_rot dims (the layout rope_kv rotates); K is assembled the same
        way, and q.k over the head is unchanged by the common permutation."""
        hp = self.hp
        H, dk, rot = hp.n_head, hp.head_dim, self.rot
        perm = np.concatenate([np.r_[h * dk + dk - rot:(h + 1) * dk, h * dk:h * dk + dk - rot] for h in range(H)])

        def qw_rows(name):
            t = T[name]
            raw, (N, K), gt = _raw2d(t)
            rows = raw.reshape(N, -1)[perm].reshape(-1)
            return ops.QWeight.from_raw(np.ascontiguousarray(rows), gt, (N, K), self.device)

        m = {"kv_a": qw(b + "attn_kv_a_mqa.weight"), "kv_a_norm": f32(b + "attn_kv_a_norm.weight"),
             "kv_b": qw(b + "attn_kv_b.weight")}
        if hp.q_lora_rank:
            m["q_a"] = qw(b + "attn_q_a.weight")
            m["q_a_norm"] = f32(b + "attn_q_a_norm.weight")
            m["q_b"] = qw_rows(b + "attn_q_b.weight")
        else:
            m["q"] = qw_rows(b + "attn_q.weight")
        return m

    def _mla_qkv(self, L: Layer, xn: torch.Tensor) -> ops.Partial:
        """q | k | v rows for rope_kv / attention from the latent projections: q per head
        [rope | nope]; c = RMSNorm(x Wkv_a[:rank]), k_pe = x Wkv_a[rank:] (one head, shared);
        [k_nope | v] = c Wkv_b per head; K = [k_pe | k_nope], V = [v | 0] (padded to the key width)."""
        hp = self.hp
        m = L.mla
        T = xn.shape[0]
        H, dk, dv, rot, r = hp.n_head, hp.head_dim, hp.head_dim_v, self.rot, hp.kv_lora_rank
        eps = hp.norm_eps
        if "q" in m:
            q = ops.reduce(ops.linear(xn, m["q"]))
        else:
            qa = ops.reduce(ops.linear(xn, m["q_a"]))
            q = ops.reduce(ops.linear(ops.add_norm(qa, None, m["q_a_norm"], None, eps), m["q_b"]))
        kva = ops.reduce(ops.linear(xn, m["kv_a"]))                       # [T, rank + rot]
        c = ops.add_norm(kva[:, :r].contiguous(), None, m["kv_a_norm"], None, eps)
        kv = ops.reduce(ops.linear(c, m["kv_b"])).view(T, H, (dk - rot) + dv)
        k = torch.cat([kva[:, r:].unsqueeze(1).expand(T, H, rot), kv[:, :, :dk - rot]], -1)
        v = torch.cat([kv[:, :, dk - rot:], kv.new_zeros(T, H, dk - dv)], -1)
        return ops.Partial(torch.cat([q, k.reshape(T, H * dk), v.reshape(T, H * dk)], -1).unsqueeze(0))

    def _attn_out(self, L: Layer, a: torch.Tensor, T: int) -> ops.Partial:
        if L.mla is not None:  # drop the value padding: [T, H, dk] -> [T, H * dv]
            a = a.view(T, self.Hq, self.Dh)[:, :, :self.hp.head_dim_v].reshape(T, -1).contiguous()
        else:
            a = a.view(T, self.Hq * self.Dh)
        return self._row_parallel(a, L.wo, L.wo_bias)

    def _expert_slice(self, t, e, rows=None, cols=None):
        E = t.shape[0]
        N, K = t.shape[1], t.shape[2]
        bs, bb = GGML_BLOCK[t.ggml_type]
        per = N * K // bs * bb
        sub = type("T", (), {})()
        sub.shape, sub.ggml_type = (N, K), t.ggml_type
        sub.data = t.data[e * per:(e + 1) * per]
        raw, shape, gt = _raw2d(sub, rows, cols)
        return ops.QWeight.from_raw(raw, gt, shape, self.device)

    # --------------------------------------------------------------------------- forward
    def new_kv_cache(self, num_blocks: int, block_size: int) -> KVCache:
        return KVCache(self.hp.n_layer, num_blocks, self.Hkv, block_size, self.Dh, self.device)

    def _row_parallel_out(self, p: ops.Partial, bias) -> ops.Partial:
        if self.tp.world == 1:
            return ops.Partial(p.t, bias)
        if self._defer_ar and p.t.is_cuda and p.bias is None and p.S <= ALLREDUCE_ADD_NORM_MAX_SLABS:
            # (the fused AR + add + norm kernel takes at most 64 split-K slabs; a MoE down
            # projection's S * top-k slabs take the reduce + all-reduce path below)
            return PendingAR(p, bias)
        car = self.tp.car
        if (TP_AR_BF16 and p.t.is_cuda and p.M <= TP_AR_BF16_MAX_ROWS and car is not None
                and p.M * p.N <= max(car.max_elems, car.max_elems2)):
            # decode rows travel in bf16 (16 KiB per 8192-wide row): half the bytes
            # of the fp32 sum over xGMI; the consumer (add_norm) reads a bf16 matrix directly.
            # Only where the custom one-/two-shot all-reduce (fp32 accumulate) takes it: an RCCL
            # ring would round at every step, and prefill-size sums keep fp32 at every chunk size
            dense = ops.reduce(p, dtype=torch.bfloat16)
            self.tp.all_reduce(dense)
            return ops.Partial(dense, bias)
        dense = ops.reduce(p)
        self.tp.all_reduce(dense)
        return ops.Partial(dense.unsqueeze(0), bias)

    def _row_parallel(self, x: torch.Tensor, w, bias) -> ops.Partial:
        """x @ w^T for a row-parallel weight (its input features sharded over the TP ranks),
        summed over the ranks.  Prefill-size inputs (>= TP_OVERLAP_ROWS rows) run in row chunks:
        chunk k's all-reduce runs on the TP comm stream while chunk k+1's GEMM runs on the compute
        stream, so the ~64-128 MB prefill all-reduces over xGMI hide under the GEMMs (SURVEY
        §2.11); decode batches keep the single latency-bound call (custom one-shot AR)."""
        tp = self.tp
        T = x.shape[0]
        if tp.world == 1 or T < TP_OVERLAP_ROWS or TP_OVERLAP_CHUNKS < 2:
            return self._row_parallel_out(ops.linear(x, w), bias)
        step = -(-T // TP_OVERLAP_CHUNKS)
        step = -(-step // 64) * 64
        out = torch.empty(T, w.N, dtype=torch.float32, device=x.device)
        cuda = x.is_cuda
        if cuda:
            cs = torch.cuda.current_stream(x.device)
            comm = tp.comm_stream(x.device)
        for r0 in range(0, T, step):
            r1 = min(T, r0 + step)
            p = ops.linear(x[r0:r1], w)
            ops.reduce(p, out=out[r0:r1])
            if cuda:
                ev = torch.cuda.Event()
                ev.record(cs)
                comm.wait_event(ev)
                with torch.cuda.stream(comm):
                    tp.all_reduce(out[r0:r1])
            else:
                tp.all_reduce(out[r0:r1])
        if cuda:
            cs.wait_stream(comm)
            out.record_stream(comm)
        return ops.Partial(out.unsqueeze(0), bias)

    def _mlp(self, L: Layer, xn: torch.Tensor) -> ops.Partial:
        hp = self.hp
        if L.experts is not None:
            return self._moe(L, xn)
        F, mode = L.F or self.F, _ACT[hp.act]
        h = ops.glu_linear(xn, L.gate_up, F, mode, L.up_bias)  # decode batches: act in the GEMM epilogue
        if h is not None:
            return self._row_parallel(h, L.down, L.down_bias)
        gu = ops.linear_multi(xn, L.gate_up, bias=L.up_bias)
        d = ops.act_linear(gu, F, mode, L.down)
        return self._row_parallel_out(d, L.down_bias)

    def _moe(self, L: Layer, xn: torch.Tensor, routed=None) -> ops.Partial:
        """Mixtral sparse MoE: softmax router, top-k, renormalised weights (K16/K18), per-expert
        quantised GEMMs on the routed rows (K17), weighted scatter-add."""
        hp = self.hp
        T = xn.shape[0]
        El, base = self.E_local, self.ep_base
        if (L.moe_gu is not None and xn.is_cuda and not FUSED_ROUTER_OFF and L.experts is not None
                and T >= MOE_DENSE_MIN_T and not torch.cuda.is_current_stream_capturing()
                and not ops.moe_bs_ok(L.moe_gu, L.moe_down, T)):
            return self._moe_dense_prefill(L, xn, routed)
        if L.moe_gu is not None and xn.is_cuda and not FUSED_ROUTER_OFF:
            # any batch: one fused router launch (softmax, top-k, renorm, EP remap) feeds the
            # grouped expert GEMMs (row-chunked past 64 rows per expert); no host round trip
            # anywhere, so decode steps at every batch size capture into graphs
            k = hp.n_expert_used
            ids, wts = routed if routed is not None else ops.moe_router(
                xn, L.router, k, hp.moe_renorm, hp.expert_weights_scale, base if self.ep else 0, El if self.ep else 0)
            if ops.moe_gemv_ok(L.moe_gu, T) and ops.moe_gemv_ok(L.moe_down, T):
                # 1-2 token decode: the routed experts as int8-dot GEMVs, SwiGLU fused into the
                # down projection's prologue (no route / grouping launch, no activation launch)
                fid = ids.reshape(-1)
                gu = ops.moe_gemv(xn, L.moe_gu, fid, k, T, El)
                d = ops.moe_gemv(None, L.moe_down, fid, k, T, El, act_src=gu, act_mode=ops.ACT_SWIGLU, wts=wts)
                if L.shexp_down is not None:
                    d = ops.Partial((ops.reduce(d) + self._shared_expert(L, xn)).unsqueeze(0))
                return self._row_parallel_out(d, None)
            order, off = ops.moe_route(ids, El + 1 if self.ep else El)
            if ops.moe_bs_ok(L.moe_gu, L.moe_down, T):
                # prefill chunks: the grouped shared-dequant-image tiles, 256 routed rows per weight
                # stream, one launch per projection for any routing (no host read of `off`)
                h = ops.moe_glu_bs(xn, L.moe_gu, order, off, k, T)
                d = ops.moe_down_bs(h, L.moe_down, order, off, k, T, wts, zero=self.ep)
            elif ops.moe32_ok(L.moe_gu, L.moe_down, T):
                # wide batch: 32x32x16 grouped tiles, SwiGLU fused into the gate|up epilogue
                h = ops.moe_glu32(xn, L.moe_gu, order, off, k, T)
                d = ops.moe_down32(h, L.moe_down, order, off, k, T, wts, zero=self.ep)
            else:
                gu = ops.moe_linear(xn, L.moe_gu, order, off, k, T)
                h = ops.act(gu, L.F or self.F, ops.ACT_SWIGLU)
                d = ops.moe_linear(h, L.moe_down, order, off, k, T, down=True, wts=wts, zero=self.ep)
            if L.shexp_down is not None:
                d = ops.Partial((ops.reduce(d) + self._shared_expert(L, xn)).unsqueeze(0))
            return self._row_parallel_out(d, None)
        logits = xn.float() @ L.router.t()                       # [T, E]
        w, idx = torch.topk(torch.softmax(logits, -1), hp.n_expert_used, -1)
        if hp.moe_renorm:
            w = w / w.sum(-1, keepdim=True)
        if hp.expert_weights_scale != 1.0:
            w = w * hp.expert_weights_scale
        if self.ep:
            # expert ids of this rank -> 0..El-1; tokens' other picks -> El (a group nobody runs)
            loc = idx - base
            idx_l = torch.where((loc >= 0) & (loc < El), loc, torch.full_like(loc, El))
        else:
            idx_l = idx
        if L.moe_gu is not None and xn.is_cuda:
            # graph-capturable grouped path: device routing, one weight stream per active expert,
            # routing-weighted outputs land as extra slabs summed by the next kernel
            k = hp.n_expert_used
            order, off = ops.moe_route(idx_l.to(torch.int32), El + 1 if self.ep else El)
            gu = ops.moe_linear(xn, L.moe_gu, order, off, k, T)
            h = ops.act(gu, L.F or self.F, ops.ACT_SWIGLU)
            d = ops.moe_linear(h, L.moe_down, order, off, k, T, down=True,
                               wts=w.reshape(-1).float().contiguous(), zero=self.ep)
            if L.shexp_down is not None:
                d = ops.Partial((ops.reduce(d) + self._shared_expert(L, xn)).unsqueeze(0))
            return self._row_parallel_out(d, None)
        out = torch.zeros(T, hp.n_embd, dtype=torch.float32, device=xn.device)
        flat_e = idx_l.reshape(-1)
        flat_t = torch.arange(T, device=xn.device).repeat_interleave(hp.n_expert_used)
        flat_w = w.reshape(-1)
        with ops.blas_tuning_paused():  # per-expert M varies every step: never tune those shapes
            for e, (gate_up, down) in enumerate(L.experts):
                sel = (flat_e == e).nonzero(as_tuple=True)[0]
                if sel.numel() == 0:
                    continue
                rows = flat_t[sel]
                xe = xn.index_select(0, rows).contiguous()
                gu = ops.linear_multi(xe, gate_up)
                h = ops.act(gu, L.F or self.F, ops.ACT_SWIGLU)
                d = ops.reduce(ops.linear(h, down))
                out.index_add_(0, rows, d * flat_w[sel].unsqueeze(1))
        if L.shexp_down is not None:
            out += self._shared_expert(L, xn)
        self.tp.all_reduce(out)
        return ops.Partial(out.unsqueeze(0))

    def _moe_dense_prefill(self, L: Layer, xn: torch.Tensor, routed=None) -> ops.Partial:
        """Prefill-sized MoE: device routing (fused router + grouping), ONE host read of the
        per-expert row offsets, then per expert a dense gate|up GEMM over its gathered rows, the
        SwiGLU, the down GEMM, and a routing-weighted index_add back to the tokens (two
        contributions per row for top-2 -- order-independent in fp32)."""
        hp = self.hp
        T = xn.shape[0]
        k = hp.n_expert_used
        El, base = self.E_local, self.ep_base
        ids, wts = routed if routed is not None else ops.moe_router(
            xn, L.router, k, hp.moe_renorm, hp.expert_weights_scale, base if self.ep else 0, El if self.ep else 0)
        order, off = ops.moe_route(ids, El + 1 if self.ep else El)
        off_h = off.cpu().tolist()
        order_l = order.long()
        tok = order_l // k
        xs = xn.index_select(0, tok)                         # [T*k, D], grouped by expert
        wsel = wts.reshape(-1).float().index_select(0, order_l)
        out = torch.zeros(T, hp.n_embd, dtype=torch.float32, device=xn.device)
        with ops.blas_tuning_paused():  # per-expert row counts vary every chunk: never tune them
            for e in range(El):
                r0, r1 = off_h[e], off_h[e + 1]
                if r1 <= r0:
                    continue
                gate_up, down = L.experts[e]
                gu = ops.linear_multi(xs[r0:r1], gate_up)
                h = ops.act(gu, L.F or self.F, ops.ACT_SWIGLU)
                d = ops.reduce(ops.linear(h, down))
                out.index_add_(0, tok[r0:r1], d * wsel[r0:r1].unsqueeze(1))
        if L.shexp_down is not None:
            out += self._shared_expert(L, xn)
        self.tp.all_reduce(out)
        return ops.Partial(out.unsqueeze(0))

    def _shared_expert(self, L: Layer, xn: torch.Tensor) -> torch.Tensor:
        """Shared expert(s): down(silu(gate x) * up x) on this rank's F slice, fp32 [T, D]; scaled by
        sigmoid(x . g_shexp) for Qwen2-MoE, unscaled for DeepSeek-V2."""
        gu = ops.linear_multi(xn, L.shexp_gate_up)
        sh = ops.reduce(ops.act_linear(gu, self.hp.n_ff_shexp // self.tp.world, ops.ACT_SWIGLU, L.shexp_down))
        if L.shexp_gate is None:
            return sh
        return sh * torch.sigmoid(xn.float() @ L.shexp_gate).unsqueeze(1)

    def _add_norm(self, res, o, w, b, eps, nm):
        """ops.add_norm, or -- for a deferred TP all-reduce -- the fused all-reduce + add + norm."""
        if isinstance(o, PendingAR):
            return self.tp.car.add_norm(o.part, o.bias, res, w, b, eps, nm)
        return ops.add_norm(res, o, w, b, eps, nm)

    def _post_attn(self, i: int, L: Layer, xn: torch.Tensor, res: torch.Tensor, o: ops.Partial,
                   defer_to: Optional[torch.Tensor] = None):
        """Residual + norm around the MLP of layer i; returns the next layer's normed input -- or,
        with defer_to (batch-1/2 decode, next consumer = the fused q|k|v GEMV), an ops.NormIn that
        the next GEMV applies in its prologue, the updated residual landing in defer_to."""
        hp = self.hp
        eps, nm = hp.norm_eps, self.norm_mode
        nxt = self.layers[i + 1] if i + 1 < len(self.layers) else None
        nw = nxt.attn_norm if nxt is not None else self.out_norm
        nb = nxt.attn_norm_b if nxt is not None else self.out_norm_b
        if hp.parallel_residual:
            f = self._mlp(L, xn)
            ops.add_norm(res, o, nw, nb, eps, nm, want_out=False)
            return ops.add_norm(res, f, nw, nb, eps, nm)
        if L.post_attn_norm is not None:
            o = self._post_norm(o, L.post_attn_norm)
        fused = None
        if (L.experts is not None and L.moe_gu is not None and res.is_cuda and not FUSED_ROUTER_OFF
                and not isinstance(o, PendingAR)):
            # sparse MoE: the router rides on the add_norm launch (ops.add_norm_router)
            k = hp.n_expert_used
            fused = ops.add_norm_router(res, o, L.ffn_norm, L.ffn_norm_b, eps, nm, L.router, k, hp.moe_renorm,
                                        hp.expert_weights_scale, self.ep_base if self.ep else 0,
                                        self.E_local if self.ep else 0)
        if fused is not None:
            xn = fused[0]
            f = self._moe(L, xn, routed=fused[1:])
        else:
            xn = self._add_norm(res, o, L.ffn_norm, L.ffn_norm_b, eps, nm)
            f = self._mlp(L, xn)
        if L.post_ffw_norm is not None:
            f = self._post_norm(f, L.post_ffw_norm)
        if (defer_to is not None and nxt is not None and nm == 0 and isinstance(f, ops.Partial)
                and ops.norm_in_ok(res, f, nw, nb)):
            return ops.NormIn(res, f, nw, eps, defer_to)
        return self._add_norm(res, f, nw, nb, eps, nm)

    def _post_norm(self, p: ops.Partial, w: torch.Tensor) -> ops.Partial:
        """RMSNorm(p) * w as an fp32 partial (Gemma-2's post-attention / post-FFW norms)."""
        T = p.M
        zero = torch.zeros(T, self.hp.n_embd, dtype=torch.float32, device=p.t.device)
        y = torch.empty_like(zero)
        ops.add_norm(zero, p, w, None, self.hp.norm_eps, self.norm_mode, out_f32=y)
        return ops.Partial(y.unsqueeze(0))

    def forward(self, fb: ForwardBatch, kv: KVCache, attn_workspace=None, return_hidden: bool = False,
                local_logits: bool = False) -> torch.Tensor:
        """Returns fp32 logits [R, V] for the rows selected by fb.logits_idx (or, with
        return_hidden, the final-norm hidden states [T, D]).  local_logits: under tensor
        parallelism return this rank's vocabulary columns [R, V / world] (no all-gather; the
        caller reduces them, e.g. TPInfo.argmax_cols)."""
        hp = self.hp
        eps, nm = hp.norm_eps, self.norm_mode
        T = fb.tokens.shape[0]
        res = ops.embed(fb.tokens, self.tok_embd, hp.embed_scale)
        if fb.inject_idx is not None:
            res.index_copy_(0, fb.inject_idx, fb.inject_rows.to(res.dtype))
        L0 = self.layers[0]
        fuse_qkv = fb.decode and FUSED_QKV_ROPE and ops.qkv_rope_ok(res, self.layers[0].qkv, self.layers[0].qkv_bias,
                                                                    hp.rope_mode, self.rot, self.Dh, kv.block_size)
        # batch-1/2 decode: every layer boundary's residual-add + RMSNorm runs inside the next
        # q|k|v GEMV's prologue (ops.NormIn); the residual ping-pongs between two buffers because
        # that GEMV's workgroups read one while its first workgroup writes the other
        fuse_norm = (fuse_qkv and nm == 0 and not hp.parallel_residual
                     and ops.norm_in_ok(res, None, L0.attn_norm, L0.attn_norm_b))
        res2 = torch.empty_like(res) if fuse_norm else None
        # GPU TP decode: each layer boundary's all-reduce runs fused with its add_norm
        car = self.tp.car
        self._defer_ar = bool(fb.decode and self.tp.world > 1 and car is not None and res.is_cuda
                              and not hp.parallel_residual and hasattr(car, "supports_add_norm")
                              and car.supports_add_norm(T, res.shape[1])
                              and all(L.post_attn_norm is None and L.post_ffw_norm is None for L in self.layers))
        if fuse_norm:
            xn = ops.NormIn(res, None, L0.attn_norm, eps, None)
        else:
            xn = ops.add_norm(res, None, L0.attn_norm, L0.attn_norm_b, eps, nm)
        for i, L in enumerate(self.layers):
            if fuse_qkv:
                # batch-1/2 decode: q|k|v GEMV with RoPE + the paged K/V append in its epilogue
                q = ops.qkv_rope_dp4(xn, L.qkv, fb.pos, fb.slots, self.cos_sin, self.Hq, self.Hkv, self.Dh,
                                     kv.k[i], kv.v[i], kv.block_size)
                if isinstance(xn, ops.NormIn) and xn.res_out is not None:
                    res, res2 = xn.res_out, xn.res  # the updated residual now lives in the other buffer
                a = ops.attn_decode(q, kv.k[i], kv.v[i], fb.block_tables, fb.seq_lens, self.scale, fb.max_len,
                                    workspace=attn_workspace, softcap=hp.attn_softcap, window=L.window)
                o = self._row_parallel_out(ops.linear(a.view(T, self.Hq * self.Dh), L.wo), L.wo_bias)
                xn = self._post_attn(i, L, xn, res, o, defer_to=res2)
                continue
            qkv = self._mla_qkv(L, xn) if L.mla is not None else ops.linear_multi(xn, L.qkv, bias=L.qkv_bias)
            if fb.decode:
                # RoPE + KV append fused into the decode attention launch (rope_kv when not fusable)
                a = ops.attn_decode_rope(qkv, fb.pos, fb.slots, self.cos_sin, self.Hq, self.Hkv, self.Dh, self.rot,
                                         hp.rope_mode, kv.k[i], kv.v[i], fb.block_tables, fb.seq_lens, self.scale,
                                         fb.max_len, workspace=attn_workspace, softcap=hp.attn_softcap,
                                         window=L.window)
            else:
                q = ops.rope_kv(qkv, fb.pos, fb.slots, self.cos_sin, self.Hq, self.Hkv, self.Dh, self.rot,
                                hp.rope_mode, kv.k[i], kv.v[i], kv.block_size)
                a = ops.attn_prefill(q, kv.k[i], kv.v[i], fb.cu_q, fb.ctx_lens, fb.block_tables, self.scale,
                                     tiles=fb.tiles, softcap=hp.attn_softcap, window=L.window)
            o = self._attn_out(L, a, T)
            xn = self._post_attn(i, L, xn, res, o)
        if return_hidden:
            return xn
        rows = xn if fb.logits_idx is None else xn.index_select(0, fb.logits_idx)
        lp = ops.linear(rows.contiguous(), self.output, bias=self.out_bias)
        if lp.S == 1 and lp.bias is None:
            logits = lp.t[0]
        else:
            logits = ops.reduce(lp)
        if not local_logits:
            logits = self.tp.all_gather_cols(logits)
        if self.hp.logit_scale != 1.0:
            logits = logits * self.hp.logit_scale
        if self.hp.final_softcap:
            c = self.hp.final_softcap
            logits = torch.tanh(logits / c) * c
        return logits

    def reference_logits(self, tokens: Sequence[int]) -> torch.Tensor:
        """Plain fp32 PyTorch forward of one sequence (no paging): the numerics oracle for the
        GPU engine and for the TP tests.  Uses dequantised weights."""
        hp = self.hp
        dev = torch.device("cpu")
        t = torch.tensor(tokens, dtype=torch.long)
        Tn = len(tokens)
        # dequantised fp32 host copies are kept across calls (an oracle checks hundreds of rows;
        # re-dequantising every weight per call dominated test_headline_path_against_fp32_oracle)
        cache = self.__dict__.setdefault("_oracle_w", {})

        def deq(w):
            if w.ref is not None:
                return w.ref.cpu()
            if id(w) not in cache:
                cache[id(w)] = (w, w.materialize_bf16().float().cpu())
            return cache[id(w)][1]

        x = self.tok_embd.dequant_f32().to(dev)[t] if self.tok_embd.ref is not None else deq(self.tok_embd)[t]
        x = x * hp.embed_scale

        def norm(x, w, b):
            if self.norm_mode == 0:
                return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + hp.norm_eps) * w.cpu()
            mu = x.mean(-1, keepdim=True)
            y = (x - mu) * torch.rsqrt((x - mu).pow(2).mean(-1, keepdim=True) + hp.norm_eps) * w.cpu()
            return y + b.cpu() if b is not None else y

        cs = self.cos_sin.cpu()[:Tn]
        c, s = cs[..., 0], cs[..., 1]

        def rope(h):
            h = h.clone()
            r = self.rot
            if hp.rope_mode == 0:
                x0, x1 = h[..., 0:r:2].clone(), h[..., 1:r:2].clone()
                h[..., 0:r:2] = x0 * c[:, None] - x1 * s[:, None]
                h[..., 1:r:2] = x0 * s[:, None] + x1 * c[:, None]
            else:
                hf = r // 2
                x0, x1 = h[..., :hf].clone(), h[..., hf:r].clone()
                h[..., :hf] = x0 * c[:, None] - x1 * s[:, None]
                h[..., hf:r] = x0 * s[:, None] + x1 * c[:, None]
            return h

        Hq, Hkv, Dh = self.Hq, self.Hkv, self.Dh
        mask = torch.triu(torch.full((Tn, Tn), float("-inf")), 1)
        def rms(x, w):
            return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + hp.norm_eps) * w.cpu()

        for L in self.layers:
            h = norm(x, L.attn_norm, L.attn_norm_b)
            if L.mla is not None:  # latent attention, same [rope | nope] head layout as _mla_qkv
                m, H, dk, dv, rt, r = L.mla, hp.n_head, hp.head_dim, hp.head_dim_v, self.rot, hp.kv_lora_rank
                q = h @ deq(m["q"]).t() if "q" in m else rms(h @ deq(m["q_a"]).t(), m["q_a_norm"]) @ deq(m["q_b"]).t()
                kva = h @ deq(m["kv_a"]).t()
                kvb = (rms(kva[:, :r], m["kv_a_norm"]) @ deq(m["kv_b"]).t()).view(Tn, H, dk - rt + dv)
                kk = torch.cat([kva[:, r:].unsqueeze(1).expand(Tn, H, rt), kvb[:, :, :dk - rt]], -1)
                vv = torch.cat([kvb[:, :, dk - rt:], kvb.new_zeros(Tn, H, dk - dv)], -1)
                qkv = torch.cat([q, kk.reshape(Tn, -1), vv.reshape(Tn, -1)], -1)
            else:
                qkv = torch.cat([h @ deq(w).t() for w in L.qkv], -1)
            if L.qkv_bias is not None:
                qkv = qkv + L.qkv_bias.cpu()
            q = rope(qkv[:, :Hq * Dh].view(Tn, Hq, Dh))
            k = rope(qkv[:, Hq * Dh:(Hq + Hkv) * Dh].view(Tn, Hkv, Dh))
            v = qkv[:, (Hq + Hkv) * Dh:].view(Tn, Hkv, Dh)
            G = Hq // Hkv
            k = k.repeat_interleave(G, 1)
            v = v.repeat_interleave(G, 1)
            att = torch.einsum("qhd,khd->hqk", q, k) * self.scale
            if hp.attn_softcap:
                att = torch.tanh(att / hp.attn_softcap) * hp.attn_softcap
            att = att + mask
            if L.window:
                pos = torch.arange(Tn)
                att = att.masked_fill((pos.view(-1, 1) - pos.view(1, -1)) >= L.window, float("-inf"))
            a = torch.einsum("hqk,khd->qhd", torch.softmax(att, -1), v)
            a = a[:, :, :hp.head_dim_v].reshape(Tn, -1) if L.mla is not None else a.reshape(Tn, Hq * Dh)
            o = a @ deq(L.wo).t()
            if L.wo_bias is not None:
                o = o + L.wo_bias.cpu()
            if L.post_attn_norm is not None:
                o = norm(o, L.post_attn_norm, None)

            def mlp(hin):
                if L.experts is not None:
                    lg = hin @ L.router.cpu().t()
                    w, idx = torch.topk(torch.softmax(lg, -1), hp.n_expert_used, -1)
                    if hp.moe_renorm:
                        w = w / w.sum(-1, keepdim=True)
                    w = w * hp.expert_weights_scale
                    out = torch.zeros_like(hin)
                    for tt in range(Tn):
                        for j in range(hp.n_expert_used):
                            gu_w, dw = L.experts[int(idx[tt, j])]
                            gu = torch.cat([hin[tt:tt + 1] @ deq(ww).t() for ww in gu_w], -1)
                            ff = gu.shape[-1] // 2
                            hh = torch.nn.functional.silu(gu[:, :ff]) * gu[:, ff:]
                            out[tt] += w[tt, j] * (hh @ deq(dw).t())[0]
                    if L.shexp_down is not None:
                        gu = torch.cat([hin @ deq(ww).t() for ww in L.shexp_gate_up], -1)
                        ff = gu.shape[-1] // 2
                        sh = (torch.nn.functional.silu(gu[:, :ff]) * gu[:, ff:]) @ deq(L.shexp_down).t()
                        if L.shexp_gate is not None:
                            sh = torch.sigmoid(hin @ L.shexp_gate.cpu()).unsqueeze(1) * sh
                        out = out + sh
                    return out
                gu = torch.cat([hin @ deq(w).t() for w in L.gate_up], -1)
                if L.up_bias is not None:
                    gu = gu + L.up_bias.cpu()
                F = L.F or self.F
                if hp.act == "swiglu":
                    hh = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
                elif hp.act == "geglu":
                    hh = torch.nn.functional.gelu(gu[:, :F], approximate="tanh") * gu[:, F:]
                else:
                    hh = torch.nn.functional.gelu(gu, approximate="tanh")
                d = hh @ deq(L.down).t()
                if L.down_bias is not None:
                    d = d + L.down_bias.cpu()
                if L.post_ffw_norm is not None:
                    d = norm(d, L.post_ffw_norm, None)
                return d

            if hp.parallel_residual:
                x = x + o + mlp(h)
            else:
                x = x + o
                x = x + mlp(norm(x, L.ffn_norm, L.ffn_norm_b))
        x = norm(x, self.out_norm, self.out_norm_b)
        lg = x @ deq(self.output).t()
        if self.out_bias is not None:
            lg = lg + self.out_bias.cpu()
        lg = lg * hp.logit_scale
        if hp.final_softcap:
            lg = torch.tanh(lg / hp.final_softcap) * hp.final_softcap
        return lg
