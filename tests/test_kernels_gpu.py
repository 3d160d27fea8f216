"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op."""
import math

import numpy as np
import pytest
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, quantize

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _qw(N, K, t, seed=0, std=0.05):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((N, K)).astype(np.float32) * std
    raw = quantize(w, t)
    return ops.QWeight.from_raw(raw, t, (N, K), DEV, keep_ref=True)


def test_library_loads():
    assert ops.hip_available()
    assert ops.lib().la_sample_row_bytes() == ops.SAMPLE_ROW_DTYPE.itemsize


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.F16])
@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
def test_skinny_gemm(t, M):
    N, K = 320, 1024
    w = _qw(N, K, t)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = ops.linear(x, w, force="skinny").dense()
    ref = x.float().cpu() @ w.ref.t()
    err = (y.cpu() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


def test_skinny_gemm_splits_and_tail():
    # N not a multiple of 64, K = 14 super-blocks (split-K by 7 / 14)
    N, K, M = 200, 3584, 3
    w = _qw(N, K, GGMLType.Q4_K, seed=3)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    for S in (1, 2, 7, 14):
        out = torch.empty(S, M, N, dtype=torch.float32, device=DEV)
        rc = ops.lib().la_qgemm_skinny(w.fmt, *w.ptrs(), N, K, x.data_ptr(), K, M, S, out.data_ptr(), N, M * N,
                                       ops._stream())
        assert rc == 0
        ref = x.float().cpu() @ w.ref.t()
        assert (out.sum(0).cpu() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_gemv_dp4(t, M):
    """int8-dot decode GEMV (activations quantised per 256-block, ggml q8_K style) vs fp32:
    N off the 64-row workgroup tile, every split of K, repeated launches bit-identical."""
    N, K = 200, 3584
    w = _qw(N, K, t, seed=11)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    for S in (1, 2, 7, 14):
        out = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=DEV)
        ops.gemv_dp4(x, [w], S, out)
        err = (out.sum(0).cpu() - ref).abs().max().item()
        assert err < tol, (S, err)
        out2 = torch.empty_like(out)
        ops.gemv_dp4(x, [w], S, out2)
        assert torch.equal(out, out2)
    y = ops.linear(x, w, force="dp4").dense().cpu()
    assert (y - ref).abs().max().item() < tol


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("M", [1, 2])
def test_act_linear_fused(mode, M):
    """down(act(gate|up)) with the activation inside the dp4 GEMV prologue vs fp32 (slab source
    with S = 3 and a bias)."""
    F, N = 1024, 200
    w = _qw(N, F, GGMLType.Q6_K if mode else GGMLType.Q4_K, seed=17)
    width = 2 * F if mode == 0 else F
    slabs = torch.randn(3, M, width, device=DEV) * 0.7
    bias = torch.randn(width, device=DEV) * 0.1
    src = ops.Partial(slabs, bias)
    y = ops.act_linear(src, F, mode, w).dense().cpu()
    g = (slabs.sum(0) + bias).cpu()
    if mode == 0:
        h = torch.nn.functional.silu(g[:, :F]) * g[:, F:]
    elif mode == 1:
        h = torch.nn.functional.gelu(g, approximate="tanh")
    else:
        h = g * torch.sigmoid(1.702 * g)
    ref = h @ w.ref.t()
    assert (y - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("M", [1, 3])
def test_gemv_dp4_segments(M):
    """One launch over mixed-format weights side by side (Q4_K q|k + Q6_K v shape), plus a
    4-weight call that spills into a second launch."""
    K = 1024
    ws = [_qw(136, K, GGMLType.Q4_K, seed=13), _qw(64, K, GGMLType.Q6_K, seed=14), _qw(72, K, GGMLType.Q4_K, seed=15),
          _qw(40, K, GGMLType.Q6_K, seed=16)]
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
    for n in (2, 3, 4):
        y = ops.linear_multi(x, ws[:n], force="dp4").dense().cpu()
        assert (y - ref[:, :y.shape[1]]).abs().max().item() < 5e-2, n


def test_gemv_dp4_outlier_rows():
    """Activation rows with large outliers (post-SwiGLU-like) stay within q8 accuracy."""
    N, K = 128, 4096
    w = _qw(N, K, GGMLType.Q4_K, seed=12)
    x = torch.randn(1, K)
    x[0, ::97] *= 40.0
    x = x.to(DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    y = ops.linear(x, w, force="dp4").dense().cpu()
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("M", [65, 128, 200, 256, 300])
def test_mid_gemm(t, M):
    """Mid-M quantised MFMA GEMM (the gemm_q.hip tile kernel, heuristic tile / split-K) vs the fp32
    reference; N not a multiple of the 128-wide tile, M spanning several 128-row tiles."""
    N, K = 200, 1536
    w = _qw(N, K, t, seed=7)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = ops.linear(x, w, force="tile").dense()
    ref = x.float().cpu() @ w.ref.t()
    err = (y.cpu() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("M", [3, 100])
def test_linear_multi_mixed_formats(M):
    K = 512
    ws = [_qw(128, K, GGMLType.Q4_K, seed=4), _qw(64, K, GGMLType.Q4_K, seed=5), _qw(64, K, GGMLType.Q6_K, seed=6)]
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = ops.linear_multi(x, ws).dense().cpu()
    ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
    assert (y - ref).abs().max().item() < 5e-2


def test_fused_bf16_library_path():
    """q|k (Q4_K) + v (Q6_K) behind one bf16 matrix: one library GEMM, same result, and the
    per-weight bf16 copies become row slices of the fused buffer."""
    K = 512
    ws = [_qw(256, K, GGMLType.Q4_K, seed=7), _qw(128, K, GGMLType.Q6_K, seed=8)]
    x = torch.randn(300, K, device=DEV).to(torch.bfloat16)
    sep = ops.linear_multi(x, ws, force="blas").dense().cpu()
    fused = ops.fuse_bf16(ws)
    assert fused.shape == (384, K)
    assert ws[1].materialize_bf16().data_ptr() == fused.data_ptr() + 256 * K * 2
    one = ops.linear_multi(x, ws, force="blas").dense().cpu()
    assert (one - sep).abs().max().item() < 1e-2
    ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
    assert (one - ref).abs().max().item() < 5e-2


def test_dequant_and_large_m_linear():
    w = _qw(256, 512, GGMLType.Q4_K, seed=1)
    wb = w.materialize_bf16().float().cpu()
    assert (wb - w.ref).abs().max().item() < 1e-2
    x = torch.randn(300, 512, device=DEV).to(torch.bfloat16)
    y = ops.linear(x, w).dense().cpu()
    ref = x.float().cpu() @ w.ref.t()
    assert (y - ref).abs().max().item() < 5e-2


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("T,D", [(7, 4096), (1, 2560), (40, 4096), (3, 8192)])
def test_add_norm(mode, T, D):
    res = torch.randn(T, D, device=DEV)
    add = torch.randn(3, T, D, device=DEV)
    w = torch.rand(D, device=DEV) + 0.5
    b = torch.randn(D, device=DEV) if mode == 1 else None
    r_ref = res.cpu().clone()
    out = ops.add_norm(res, ops.Partial(add), w, b, 1e-5, mode)
    out_ref = ops.add_norm(r_ref, ops.Partial(add.cpu()), w.cpu(), None if b is None else b.cpu(), 1e-5, mode)
    assert (res.cpu() - r_ref).abs().max().item() < 1e-4
    assert (out.float().cpu() - out_ref.float()).abs().max().item() < 3e-2


@pytest.mark.parametrize("mode,Dh,rot", [(0, 128, 128), (1, 80, 32), (1, 64, 64)])
def test_rope_kv(mode, Dh, rot):
    T, Hq, Hkv, BS, nblk = 5, 8, 2, 16, 6
    qkv = torch.randn(2, T, (Hq + 2 * Hkv) * Dh, device=DEV)
    pos = torch.tensor([0, 3, 7, 100, 5], dtype=torch.int32, device=DEV)
    slots = torch.tensor([0, 17, 33, 50, -1], dtype=torch.int32, device=DEV)
    cs = ops.rope_cos_sin(256, rot, 10000.0, DEV)
    kc = torch.zeros(nblk, Hkv, BS, Dh, dtype=torch.bfloat16, device=DEV)
    vc = ops.v_pages(nblk, Hkv, BS, Dh, device=DEV)
    kr, vr = kc.cpu().clone(), vc.cpu().clone()
    q = ops.rope_kv(ops.Partial(qkv), pos, slots, cs, Hq, Hkv, Dh, rot, mode, kc, vc, BS)
    qr = ops.rope_kv(ops.Partial(qkv.cpu()), pos.cpu(), slots.cpu(), cs.cpu(), Hq, Hkv, Dh, rot, mode, kr, vr, BS)
    assert (q.float().cpu() - qr.float()).abs().max().item() < 3e-2
    assert (kc.float().cpu() - kr.float()).abs().max().item() < 3e-2
    assert (vc.float().cpu() - vr.float()).abs().max().item() < 3e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_act(mode):
    T, F = 9, 1024
    W = 2 * F if mode == 0 else F
    x = torch.randn(2, T, W, device=DEV) * 3
    y = ops.act(ops.Partial(x), F, mode)
    yr = ops.act(ops.Partial(x.cpu()), F, mode)
    assert (y.float().cpu() - yr.float()).abs().max().item() < 5e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("F", [14336, 1032, 1028])
def test_act_bf16_source(mode, F):
    """bf16 GEMM output (hipBLASLt path): F % 8 == 0 takes the 16-byte act8 kernel, else 4-wide."""
    T = 5
    W = 2 * F if mode == 0 else F
    x = (torch.randn(T, W, device=DEV) * 3).to(torch.bfloat16)
    y = ops.act(ops.Partial(x), F, mode)
    xf = x.float().cpu()
    if mode == 0:
        yr = torch.nn.functional.silu(xf[:, :F]) * xf[:, F:]
    elif mode == 1:
        yr = torch.nn.functional.gelu(xf, approximate="tanh")
    else:
        yr = xf * torch.sigmoid(1.702 * xf)
    assert (y.float().cpu() - yr).abs().max().item() < 5e-2 * max(1.0, yr.abs().max().item() / 8)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
def test_embed(t):
    w = _qw(100, 512, t)
    tok = torch.tensor([0, 5, 99, 5], dtype=torch.int32, device=DEV)
    e = ops.embed(tok, w, 2.0)
    assert (e.cpu() - w.ref[tok.cpu().long()] * 2).abs().max().item() < 1e-5


def _paged_setup(lens, Hkv, Dh, BS, seed=0):
    g = torch.Generator().manual_seed(seed)
    maxb = max((l + BS - 1) // BS for l in lens)
    nblk = sum((l + BS - 1) // BS for l in lens) + 3
    kc = torch.randn(nblk, Hkv, BS, Dh, generator=g).to(torch.bfloat16)
    vc = ops.v_from_rows(torch.randn(nblk, Hkv, BS, Dh, generator=g).to(torch.bfloat16))  # V cache layout
    perm = torch.randperm(nblk, generator=g)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32)
    c = 0
    for i, l in enumerate(lens):
        nb = (l + BS - 1) // BS
        bt[i, :nb] = perm[c:c + nb]
        c += nb
    return kc, vc, bt


@pytest.mark.parametrize("Hq,Hkv,Dh,BS", [(32, 8, 128, 32), (32, 32, 80, 32), (8, 1, 64, 16), (64, 8, 128, 32),
                                         (16, 1, 96, 64), (8, 1, 256, 32), (16, 16, 256, 32), (16, 16, 192, 32)])
@pytest.mark.parametrize("nw1", [False, True])
def test_attn_decode(Hq, Hkv, Dh, BS, nw1, monkeypatch):
    if nw1:  # single-wave workgroups (the batch-decode variant) on a small batch
        monkeypatch.setattr(ops, "DEC_NW1_MIN", 1)
    lens = [1, 37, 300, 1025]
    kc, vc, bt = _paged_setup(lens, Hkv, Dh, BS)
    q = torch.randn(len(lens), Hq, Dh).to(torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    scale = 1 / math.sqrt(Dh)
    ref = ops.attn_decode(q, kc, vc, bt, sl, scale, max(lens))
    for ml in (max(lens), 4096):  # exact bound and the graph-capture bound (many empty partitions)
        out = ops.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), scale, ml)
        assert (out.float().cpu() - ref.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("src", ["slabs", "bf16"])
@pytest.mark.parametrize("nw1", [False, True])
def test_attn_decode_fused_rope(src, nw1, monkeypatch):
    """Decode attention with RoPE + KV append fused in == rope_kv + attn_decode (outputs and the
    appended cache entries), over split-KV partitions (graph bound 4096) and a padded row."""
    Hq, Hkv, Dh, BS = 32, 8, 128, 32
    if nw1:
        monkeypatch.setattr(ops, "DEC_NW1_MIN", 1)
    lens = [1, 37, 300, 1025, 1]
    kc, vc, bt = _paged_setup(lens, Hkv, Dh, BS, seed=5)
    B, W = len(lens), (Hq + 2 * Hkv) * Dh
    g = torch.Generator().manual_seed(6)
    if src == "slabs":
        part = ops.Partial(torch.randn(3, B, W, generator=g).to(DEV), torch.randn(W, generator=g).to(DEV) * 0.1)
    else:
        part = ops.Partial(torch.randn(B, W, generator=g).to(torch.bfloat16).to(DEV))
    pos = torch.tensor([l - 1 for l in lens], dtype=torch.int32, device=DEV)
    slots = torch.tensor([int(bt[i, (l - 1) // BS]) * BS + (l - 1) % BS for i, l in enumerate(lens)],
                         dtype=torch.int32, device=DEV)
    slots[-1] = -1                                   # padded graph row: no append
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    cs = ops.rope_cos_sin(4096, Dh, 500000.0, DEV)
    outs = []
    saved = ops.FUSED_DECODE_ROPE
    for fused in (False, True):
        k, v = kc.clone().to(DEV), vc.clone().to(DEV)
        ops.FUSED_DECODE_ROPE = fused
        try:
            o = ops.attn_decode_rope(part, pos, slots, cs, Hq, Hkv, Dh, Dh, 0, k, v, bt.to(DEV), sl, 0.088, 4096)
        finally:
            ops.FUSED_DECODE_ROPE = saved
        outs.append((o.float().cpu(), k.cpu(), v.cpu()))
    (o0, k0, v0), (o1, k1, v1) = outs
    assert torch.equal(k0, k1) and torch.equal(v0, v1)
    assert (o0 - o1).abs().max().item() < 1e-2


def test_attn_decode_large_batch(monkeypatch):
    """Batch decode shapes that select single-wave workgroups by themselves: 256 sequences x 8 kv
    heads (one partition each at the graph bound) and, with the window widened, 128 x 8 (two
    partitions, merged)."""
    Hq, Hkv, Dh, BS = 32, 8, 128, 32
    for B in (256, 128):
        if B == 128:
            monkeypatch.setattr(ops, "DEC_NW1_MIN", 1024)
        assert ops.decode_waves(B, Hkv) == 1
        g = torch.Generator().manual_seed(B)
        lens = torch.randint(1, 700, (B,), generator=g).tolist()
        kc, vc, bt = _paged_setup(lens, Hkv, Dh, BS, seed=B)
        q = torch.randn(B, Hq, Dh, generator=g).to(torch.bfloat16)
        sl = torch.tensor(lens, dtype=torch.int32)
        ref = ops.attn_decode(q, kc, vc, bt, sl, 0.088, max(lens))
        out = ops.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), 0.088, 1024)
        assert (out.float().cpu() - ref.float()).abs().max().item() < 2e-2


def test_attn_decode_batch1_long():
    Hq, Hkv, Dh, BS = 32, 8, 128, 32
    lens = [3000]
    kc, vc, bt = _paged_setup(lens, Hkv, Dh, BS, seed=7)
    q = torch.randn(1, Hq, Dh).to(torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    ref = ops.attn_decode(q, kc, vc, bt, sl, 0.088, 3000)
    out = ops.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), 0.088, 3000)
    assert (out.float().cpu() - ref.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("Hq,Hkv,Dh", [(32, 8, 128), (32, 32, 80), (8, 1, 256), (16, 16, 192)])
def test_attn_prefill(Hq, Hkv, Dh):
    # (new tokens, total context) per sequence: plain prefill, prefix-cached, chunked
    qlens = [70, 5, 33]
    ctx = [70, 41, 200]
    BS = 32
    kc, vc, bt = _paged_setup(ctx, Hkv, Dh, BS, seed=1)
    T = sum(qlens)
    q = torch.randn(T, Hq, Dh).to(torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(qlens)), dtype=torch.int32)
    cl = torch.tensor(ctx, dtype=torch.int32)
    scale = 1 / math.sqrt(Dh)
    ref = ops.attn_prefill(q, kc, vc, cu, cl, bt, scale)
    out = ops.attn_prefill(q.to(DEV), kc.to(DEV), vc.to(DEV), cu.to(DEV), cl.to(DEV), bt.to(DEV), scale)
    assert (out.float().cpu() - ref.float()).abs().max().item() < 3e-2


def _params(B, **kw):
    p = np.zeros(B, dtype=ops.SAMPLE_ROW_DTYPE)
    p["temp"] = kw.get("temp", 0.0)
    p["top_p"] = kw.get("top_p", 1.0)
    p["min_p"] = kw.get("min_p", 0.0)
    p["typical_p"] = 1.0
    p["tfs_z"] = 1.0
    p["top_k"] = kw.get("top_k", 0)
    p["mirostat"] = kw.get("mirostat", 0)
    p["tau"] = 5.0
    p["eta"] = 0.1
    p["seed"] = np.arange(B) + 1
    p["counter"] = 0
    return p


def test_sample_greedy():
    B, V = 6, 128256
    l = torch.randn(B, V, device=DEV)
    t = ops.sample(l, _params(B))
    assert torch.equal(t.cpu().long(), l.argmax(-1).cpu())


@pytest.mark.parametrize("V", [128256, 32003, 4099])
def test_sample_greedy_ties_and_tails(V):
    """Batched argmax loads (clamped tail indices): ties resolve to the lowest index, and the
    maximum may sit in the last float4 or in the unaligned scalar tail."""
    B = 4
    l = torch.randn(B, V, device=DEV)
    l[0, 17] = l[0, V - 1] = 50.0          # tie: lowest index wins
    l[1, V - 1] = 60.0                     # max in the clamped last element
    l[2, (V // 4) * 4 - 1] = 70.0          # max in the last aligned float4
    t = ops.sample(l, _params(B)).cpu().long()
    assert t.tolist()[:3] == [17, V - 1, (V // 4) * 4 - 1]
    assert int(t[3]) == int(l[3].argmax())
    # unaligned row base (ld odd): scalar path only
    l2 = torch.randn(2, V + 1, device=DEV)[:, 1:]
    t2 = ops.sample(l2, _params(2)).cpu().long()
    assert torch.equal(t2, l2.argmax(-1).cpu())


def test_sample_topk1_equals_greedy():
    B, V = 4, 32000
    l = torch.randn(B, V, device=DEV)
    t = ops.sample(l, _params(B, temp=0.8, top_k=1))
    assert torch.equal(t.cpu().long(), l.argmax(-1).cpu())


def test_sample_respects_topk_topp():
    B, V = 256, 5000
    l = torch.randn(B, V, device=DEV) * 3
    p = _params(B, temp=1.0, top_k=40, top_p=0.9, min_p=0.05)
    for c in range(3):
        p["counter"] = c
        t = ops.sample(l, p).cpu().long()
        top40 = torch.topk(l.cpu(), 40, -1).indices
        assert all(int(t[b]) in set(top40[b].tolist()) for b in range(B))


def test_sample_distribution():
    # temperature sampling over 4 tokens must follow softmax
    B, V = 4096, 4
    base = torch.tensor([2.0, 1.0, 0.0, -1.0])
    l = base.repeat(B, 1).to(DEV)
    p = _params(B, temp=1.0)
    t = ops.sample(l, p).cpu()
    freq = torch.bincount(t.long(), minlength=4).float() / B
    assert (freq - torch.softmax(base, 0)).abs().max().item() < 0.03


def test_sample_mirostat():
    B, V = 8, 32000
    l = torch.randn(B, V, device=DEV) * 4
    mu = torch.full((B,), 10.0, device=DEV)
    p = _params(B, temp=1.0, mirostat=2)
    t = ops.sample(l, p, mu=mu).cpu()
    assert ((t >= 0) & (t < V)).all()
    assert not torch.allclose(mu.cpu(), torch.full((B,), 10.0))


def test_penalties():
    B, V = 3, 1000
    l = torch.randn(B, V)
    hist = torch.tensor([[1, 2, 2, -1], [5, 5, 5, 5], [7, -1, -1, -1]], dtype=torch.int32)
    hl = torch.tensor([3, 4, 1], dtype=torch.int32)
    pen = torch.tensor([[1.1, 0.1, 0.2]] * 3)
    ref = ops.penalties(l.clone(), hist, hl, pen)
    out = ops.penalties(l.to(DEV), hist.to(DEV), hl.to(DEV), pen.to(DEV))
    assert (out.cpu() - ref).abs().max().item() < 1e-5


def test_logit_bias_kernel():
    B, V, cap = 4, 1000, 32
    lg = torch.randn(B, V, device=DEV)
    ref = lg.clone().cpu()
    rows = torch.zeros(cap, dtype=torch.int32)
    cols = torch.zeros(cap, dtype=torch.int32)
    vals = torch.zeros(cap, dtype=torch.float32)
    ent = [(0, 5, 1.5), (3, 999, -math.inf), (1, 0, -2.0), (1, 0, 0.5)]
    for i, (r, c, v) in enumerate(ent):
        rows[i], cols[i], vals[i] = r, c, v
        ref[r, c] += v
    cnt = torch.tensor([len(ent)], dtype=torch.int32)
    ops.logit_bias(lg, rows.to(DEV), cols.to(DEV), vals.to(DEV), cnt.to(DEV))
    assert torch.equal(lg.cpu(), ref)


def test_decode_advance_kernel():
    B, MB, BS, K = 5, 4, 16, 3
    bt = torch.randint(0, 100, (B, MB), dtype=torch.int32)
    pos = torch.tensor([3, 15, 31, 0, 7], dtype=torch.int32)
    slots = (bt[torch.arange(B), pos.long() // BS] * BS + pos % BS).to(torch.int32)
    slots[3] = -1  # padding row
    lens = pos + 1
    tok = torch.zeros(B, dtype=torch.int32)
    prm = np.zeros(B, dtype=ops.SAMPLE_ROW_DTYPE)
    prm["counter"] = [10, 11, 12, 13, 14]
    nxt = torch.tensor([7, 8, 9, 10, 11], dtype=torch.int32)
    hist = torch.zeros(K, B, dtype=torch.int32)
    step = torch.zeros(1, dtype=torch.int32)
    st_cpu = [x.clone() for x in (tok, pos, lens, slots, hist, step)]
    prm_cpu = torch.from_numpy(prm.view(np.uint8).copy())
    ops.decode_advance(nxt, *st_cpu[:4], bt, BS, st_cpu[4], st_cpu[5], prm_cpu)
    g = [x.to(DEV) for x in (tok, pos, lens, slots, hist, step)]
    prm_dev = torch.from_numpy(prm.view(np.uint8).copy()).to(DEV)
    ops.decode_advance(nxt.to(DEV), *g[:4], bt.to(DEV), BS, g[4], g[5], prm_dev)
    for a, b in zip(g, st_cpu):
        assert torch.equal(a.cpu(), b)
    assert np.array_equal(prm_dev.cpu().numpy().view(ops.SAMPLE_ROW_DTYPE)["counter"],
                          prm_cpu.numpy().view(ops.SAMPLE_ROW_DTYPE)["counter"])
    assert int(g[5].item()) == 1 and list(g[4][0].cpu()) == [7, 8, 9, 10, 11]


@pytest.mark.parametrize("T,skew", [(1, False), (5, False), (33, False), (100, False), (256, False), (300, False),
                                    (300, True), (256, True)])
def test_moe_grouped_gemm(T, skew):
    """Grouped expert GEMM at decode and wide / prefill batch sizes (T > 64: row-chunked grid, the
    row tile sized for a balanced router's expected rows); skew: every token picks experts 0 and
    1, so two experts take T rows each (several row chunks) and the others none."""
    E, topk, D, F = 8, 2, 512, 768
    gu = [_qw(2 * F, D, GGMLType.Q4_K, seed=10 + e) for e in range(E)]
    dn = [_qw(D, F, GGMLType.Q6_K, seed=30 + e) for e in range(E)]
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    x = torch.randn(T, D, device=DEV).to(torch.bfloat16)
    if skew:
        ids = torch.tensor([[0, 1]] * T, dtype=torch.int32, device=DEV)
    else:
        ids = torch.stack([torch.randperm(E)[:topk] for _ in range(T)]).to(torch.int32).to(DEV)
    wts = torch.rand(T, topk, device=DEV)
    order, off = ops.moe_route(ids, E)
    o = order.cpu().tolist()
    assert sorted(o) == list(range(T * topk))
    idc = ids.cpu().view(-1).long()
    offc = off.cpu().tolist()
    for e in range(E):  # grouped by expert, stable (increasing pair id) inside each group
        grp = o[offc[e]:offc[e + 1]]
        assert grp == sorted(grp) and all(int(idc[p]) == e for p in grp)
    y = ops.moe_linear(x, mg, order, off, topk, T).dense().cpu()          # [T*topk, 2F]
    xc = x.float().cpu()
    ref = torch.stack([xc[p // topk] for p in range(T * topk)])
    ref = torch.stack([ref[p] @ gu[int(idc[p])].ref.t() for p in range(T * topk)])
    assert (y - ref).abs().max() < 2e-2 * max(1.0, ref.abs().max())
    h = torch.randn(T * topk, F, device=DEV).to(torch.bfloat16)
    z = ops.moe_linear(h, md, order, off, topk, T, down=True, wts=wts.reshape(-1).contiguous()).dense()  # [T, D]
    hc, wc = h.float().cpu(), wts.cpu().view(-1)
    ref = torch.zeros(T, D)
    for p in range(T * topk):
        ref[p // topk] += float(wc[p]) * (hc[p] @ dn[int(idc[p])].ref.t())
    assert (z.cpu() - ref).abs().max() < 2e-2 * max(1.0, ref.abs().max())


def test_moe_route_skewed_large():
    """Every pair on one expert (the row-chunk grid's worst case) and 4096 pairs over 64 experts."""
    for T, topk, E in ((200, 1, 8), (2048, 2, 64)):
        ids = (torch.zeros(T, topk, dtype=torch.int32) if E == 8 else
               torch.randint(0, E, (T, topk), dtype=torch.int32))
        order, off = ops.moe_route(ids.to(DEV), E)
        ref = torch.sort(ids.view(-1).long(), stable=True).indices
        assert torch.equal(order.cpu().long(), ref)
        assert off.cpu().tolist() == [0] + torch.bincount(ids.view(-1).long(), minlength=E).cumsum(0).tolist()


@pytest.mark.parametrize("M", [1, 2])
def test_qkv_rope_dp4_fused(M):
    """q|k|v decode GEMV with RoPE + paged K/V append in its epilogue vs the unfused GEMV + rope_kv
    (Llama-3 head shape, Q4_K q|k + Q6_K v segments; token 1 of M=2 has no cache slot)."""
    Hq, Hkv, Dh, BS, K, nblk = 8, 2, 128, 32, 2048, 4
    qk = _qw((Hq + Hkv) * Dh, K, GGMLType.Q4_K, seed=31)
    v = _qw(Hkv * Dh, K, GGMLType.Q6_K, seed=32)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    cs = ops.rope_cos_sin(512, Dh, 500000.0, DEV)
    pos = torch.tensor([37, 200][:M], dtype=torch.int32, device=DEV)
    slots = torch.tensor([45, -1][:M], dtype=torch.int32, device=DEV)
    kc, vc = torch.zeros(nblk, Hkv, BS, Dh, dtype=torch.bfloat16, device=DEV), ops.v_pages(nblk, Hkv, BS, Dh, device=DEV)
    q = ops.qkv_rope_dp4(x, [qk, v], pos, slots, cs, Hq, Hkv, Dh, kc, vc, BS)
    kr, vr = torch.zeros_like(kc), torch.zeros_like(vc)
    qkv = ops.linear_multi(x, [qk, v], force="dp4")
    qr = ops.rope_kv(qkv, pos, slots, cs, Hq, Hkv, Dh, Dh, 0, kr, vr, BS)
    tol = 2e-2 * max(1.0, qr.float().abs().max().item())
    assert (q.float() - qr.float()).abs().max().item() < tol
    assert (kc.float() - kr.float()).abs().max().item() < tol
    assert (vc.float() - vr.float()).abs().max().item() < tol
    assert kc.abs().sum().item() > 0 and vc.abs().sum().item() > 0


@pytest.mark.parametrize("M,S", [(1, 0), (1, 3), (2, 8), (2, 11)])
def test_qkv_rope_dp4_fused_norm(M, S, monkeypatch):
    """The layer-boundary residual-add + RMSNorm folded into the fused q|k|v GEMV's prologue
    (ops.NormIn, gemv_dp4.hip GV_NORM) vs add_norm + the same GEMV: q, the appended K/V, and the
    updated residual (written to the other buffer; S = 0: no add, nothing written)."""
    Hq, Hkv, Dh, BS, K, nblk = 8, 2, 128, 32, 4096, 4
    qk = _qw((Hq + Hkv) * Dh, K, GGMLType.Q4_K, seed=33)
    v = _qw(Hkv * Dh, K, GGMLType.Q6_K, seed=34)
    g = torch.Generator().manual_seed(5)
    res = (torch.randn(M, K, generator=g) * 2).to(DEV)
    add = ops.Partial((torch.randn(S, M, K, generator=g) * 0.5).to(DEV)) if S else None
    w = (1 + 0.1 * torch.randn(K, generator=g)).to(DEV)
    cs = ops.rope_cos_sin(512, Dh, 500000.0, DEV)
    pos = torch.tensor([37, 200][:M], dtype=torch.int32, device=DEV)
    slots = torch.tensor([45, 77][:M], dtype=torch.int32, device=DEV)
    kc, vc = torch.zeros(nblk, Hkv, BS, Dh, dtype=torch.bfloat16, device=DEV), ops.v_pages(nblk, Hkv, BS, Dh, device=DEV)
    res_out = torch.full_like(res, float("nan")) if S else None
    nin = ops.NormIn(res.clone(), add, w, 1e-5, res_out)
    monkeypatch.setattr(ops, "GEMV_NORM", True)  # off by default (measured neutral), tested here
    assert ops.norm_in_ok(nin.res, add, w, None)
    q = ops.qkv_rope_dp4(nin, [qk, v], pos, slots, cs, Hq, Hkv, Dh, kc, vc, BS)
    r2 = res.clone()
    xn = ops.add_norm(r2, add, w, None, 1e-5, 0)
    kr, vr = torch.zeros_like(kc), torch.zeros_like(vc)
    qr = ops.qkv_rope_dp4(xn, [qk, v], pos, slots, cs, Hq, Hkv, Dh, kr, vr, BS)
    torch.cuda.synchronize()
    assert torch.equal(nin.res, res), "the input residual must not be written"
    if S:
        assert torch.allclose(res_out, r2, rtol=1e-6, atol=1e-5)
    # x differs only by the bf16 rounding of xn on the unfused path (int8 image of the same values)
    tol = 2e-2 * max(1.0, qr.float().abs().max().item())
    assert (q.float() - qr.float()).abs().max().item() < tol
    assert (kc.float() - kr.float()).abs().max().item() < tol
    assert (vc.float() - vr.float()).abs().max().item() < tol
    # and against the fp32 reference of the whole op
    x32 = r2.cpu()
    x32 = x32 * torch.rsqrt(x32.pow(2).mean(-1, keepdim=True) + 1e-5) * w.cpu()
    ref = torch.cat([x32 @ qk.ref.t(), x32 @ v.ref.t()], -1)[:, :Hq * Dh].view(M, Hq, Dh)
    c, s_ = cs.cpu()[pos.long().cpu()][..., 0], cs.cpu()[pos.long().cpu()][..., 1]
    r0, r1 = ref[..., 0::2].clone(), ref[..., 1::2].clone()
    ref[..., 0::2] = r0 * c[:, None] - r1 * s_[:, None]
    ref[..., 1::2] = r0 * s_[:, None] + r1 * c[:, None]
    rel = (q.float().cpu() - ref).norm() / ref.norm()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("T", [1, 5])
def test_moe_grouped_gemm_expert_parallel(T):
    """Expert-parallel grouping: this rank holds experts 0..El-1; picks of other ranks' experts are
    routed to the extra group El, never computed, and read as 0 in the zero-initialised combine."""
    El, topk, D, F = 4, 2, 512, 768
    gu = [_qw(2 * F, D, GGMLType.Q4_K, seed=50 + e) for e in range(El)]
    dn = [_qw(D, F, GGMLType.Q6_K, seed=60 + e) for e in range(El)]
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    x = torch.randn(T, D, device=DEV).to(torch.bfloat16)
    ids = torch.stack([torch.randperm(2 * El)[:topk] for _ in range(T)]).to(torch.int32)  # global ids 0..2El-1
    ids_l = torch.where(ids < El, ids, torch.full_like(ids, El)).to(DEV)
    wts = torch.rand(T, topk, device=DEV)
    order, off = ops.moe_route(ids_l, El + 1)
    gup = ops.moe_linear(x, mg, order, off, topk, T)
    h = torch.randn(T * topk, F, device=DEV).to(torch.bfloat16)
    z = ops.moe_linear(h, md, order, off, topk, T, down=True, wts=wts.reshape(-1).contiguous(), zero=True).dense()
    ref = torch.zeros(T, D)
    for p in range(T * topk):
        t, _ = divmod(p, topk)
        e = int(ids.view(-1)[p])
        if e < El:
            ref[t] += float(wts.view(-1)[p]) * (h[p].float().cpu() @ dn[e].ref.t())
            r_gu = x[t].float().cpu() @ gu[e].ref.t()
            assert (gup.dense()[p].cpu() - r_gu).abs().max() < 2e-2 * max(1.0, r_gu.abs().max())
    assert (z.cpu() - ref).abs().max() < 2e-2 * max(1.0, ref.abs().max())


@pytest.mark.parametrize("Dh", [128, 256])
def test_attn_softcap_window(Dh):
    """Gemma-2 attention transforms on the GPU kernels (decode incl. split-KV partitions, and
    prefill over a prefix-cached context) vs the CPU references: cap * tanh(s / cap) and a
    sliding window shorter than the context."""
    Hq, Hkv, BS, cap, win = 8, 2, 32, 50.0 / 8, 100
    lens = [37, 300, 1025]
    kc, vc, bt = _paged_setup(lens, Hkv, Dh, BS, seed=9)
    g = torch.Generator().manual_seed(10)
    q = (torch.randn(len(lens), Hq, Dh, generator=g) * 3).to(torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32)
    ref = ops.attn_decode(q, kc, vc, bt, sl, 0.088, max(lens), softcap=cap, window=win)
    for ml in (max(lens), 4096):
        out = ops.attn_decode(q.to(DEV), kc.to(DEV), vc.to(DEV), bt.to(DEV), sl.to(DEV), 0.088, ml, softcap=cap,
                              window=win)
        assert (out.float().cpu() - ref.float()).abs().max().item() < 2e-2
    qlens, ctx = [70, 5, 150], [70, 41, 300]
    kc, vc, bt = _paged_setup(ctx, Hkv, Dh, BS, seed=11)
    qp = (torch.randn(sum(qlens), Hq, Dh, generator=g) * 3).to(torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(qlens)), dtype=torch.int32)
    cl = torch.tensor(ctx, dtype=torch.int32)
    ref = ops.attn_prefill(qp, kc, vc, cu, cl, bt, 0.088, softcap=cap, window=win)
    out = ops.attn_prefill(qp.to(DEV), kc.to(DEV), vc.to(DEV), cu.to(DEV), cl.to(DEV), bt.to(DEV), 0.088,
                           softcap=cap, window=win)
    assert (out.float().cpu() - ref.float()).abs().max().item() < 3e-2



@pytest.mark.parametrize("M", [1, 2])
def test_gemv_dp4_q8_0_mixed_groups_and_rope(M):
    """Q8_0 weights never share a launch with K-quants (a Q8_0 q|k|v next to a Q6_K weight splits
    into homogeneous launches), and the q|k|v + RoPE + KV-append launch runs on Q8_0."""
    K = 1024
    ws = [_qw(96, K, GGMLType.Q8_0, seed=21), _qw(64, K, GGMLType.Q6_K, seed=22), _qw(40, K, GGMLType.Q8_0, seed=23)]
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = ops.linear_multi(x, ws, force="dp4").dense().cpu()
    ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
    assert (y - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())
    Hq, Hkv, Dh, BS, K2, nblk = 8, 2, 128, 32, 2048, 4
    qkv = _qw((Hq + 2 * Hkv) * Dh, K2, GGMLType.Q8_0, seed=24)
    x2 = torch.randn(M, K2, device=DEV).to(torch.bfloat16)
    cs = ops.rope_cos_sin(512, Dh, 500000.0, DEV)
    pos = torch.tensor([37, 200][:M], dtype=torch.int32, device=DEV)
    slots = torch.tensor([45, 3][:M], dtype=torch.int32, device=DEV)
    kc, vc = torch.zeros(nblk, Hkv, BS, Dh, dtype=torch.bfloat16, device=DEV), ops.v_pages(nblk, Hkv, BS, Dh, device=DEV)
    assert ops.qkv_rope_ok(x2, [qkv], None, 0, Dh, Dh, BS)
    q = ops.qkv_rope_dp4(x2, [qkv], pos, slots, cs, Hq, Hkv, Dh, kc, vc, BS)
    kr, vr = torch.zeros_like(kc), torch.zeros_like(vc)
    qr = ops.rope_kv(ops.linear(x2, qkv, force="skinny"), pos, slots, cs, Hq, Hkv, Dh, Dh, 0, kr, vr, BS)
    tol = 3e-2 * max(1.0, qr.float().abs().max().item())
    assert (q.float() - qr.float()).abs().max().item() < tol
    assert (kc.float() - kr.float()).abs().max().item() < tol and (vc.float() - vr.float()).abs().max().item() < tol


@pytest.mark.parametrize("E,k,renorm,scale,ep", [(8, 2, True, 1.0, None), (60, 4, False, 1.0, None),
                                                 (64, 6, False, 16.0, None), (8, 2, True, 1.0, (4, 4))])
def test_moe_router_fused(E, k, renorm, scale, ep):
    """Fused decode router (moe.hip) vs softmax / top-k / renorm / scale / EP remap in fp32 torch."""
    torch.manual_seed(E + k)
    T, D = 5, 4096
    xn = (torch.randn(T, D, device="cuda") * 0.5).to(torch.bfloat16)
    router = torch.randn(E, D, device="cuda") * 0.05
    base, local = ep if ep else (0, 0)
    ids, wts = ops.moe_router(xn, router, k, renorm, scale, base, local)
    torch.cuda.synchronize()
    p = torch.softmax(xn.float() @ router.t(), -1)
    w_ref, i_ref = torch.topk(p, k, -1)
    if renorm:
        w_ref = w_ref / w_ref.sum(-1, keepdim=True)
    w_ref = w_ref * scale
    L = local or E
    loc = i_ref - base
    i_ref = torch.where((loc >= 0) & (loc < L), loc, torch.full_like(loc, L))
    gap = (torch.sort(p, -1, descending=True).values[:, k - 1] - torch.sort(p, -1, descending=True).values[:, k])
    for t in range(T):
        if float(gap[t]) < 1e-4:
            continue  # a near-tie at the k-th expert may resolve either way
        assert sorted(ids[t].tolist()) == sorted(i_ref[t].tolist())
        got = dict(zip(ids[t].tolist(), wts.view(T, k)[t].tolist()))
        for e, wv in zip(i_ref[t].tolist(), w_ref[t].tolist()):
            if e != L:  # remote experts' weights are not compared (their rows are skipped)
                assert abs(got[e] - wv) < 1e-4 * max(1.0, scale)


@pytest.mark.parametrize("pinpoints", [None, [112, 56, 56, 112, 112, 112]])
def test_clip_image_preprocess_kernel_matches_pil(tmp_path, pinpoints):
    """K26 on the device (ops/csrc/image.hip): PIL-exact BICUBIC resize (same coefficient tables,
    22-bit fixed point, uint8 horizontal pass), centre crop or anyres letterbox with the mean-colour
    fill, normalisation and tiling equal the PIL host path for images of several sizes."""
    import io

    import numpy as np
    from PIL import Image

    from localai_amd.models import synth
    from localai_amd.models.clip import ClipVision
    mm = synth.write_mmproj(str(tmp_path / "mm.gguf"), out_dim=64, dim=64, n_layer=1, heads=4, ffn=128,
                            image_size=56, patch=14, pinpoints=pinpoints)
    cv = ClipVision(mm, torch.device("cuda:0"))
    rng = np.random.default_rng(0)
    for (w, h) in [(64, 48), (300, 120), (57, 203), (56, 56), (500, 333)]:
        a = (rng.random((h, w, 3)) * 255).astype(np.uint8)
        buf = io.BytesIO()
        Image.fromarray(a).save(buf, format="PNG")
        dev, lay_d = cv.preprocess(buf.getvalue())
        host, lay_h = cv._preprocess_host(Image.fromarray(a))
        assert lay_d == lay_h and tuple(dev.shape) == tuple(host.shape), (w, h)
        assert float((dev.cpu() - host).abs().max()) < 1e-5, (w, h)
    emb_d = cv.embed_image(buf.getvalue())
    import os
    os.environ["LOCALAI_AMD_CLIP_HOST_PREPROC"] = "1"
    try:
        emb_h = cv.embed_image(buf.getvalue())
    finally:
        del os.environ["LOCALAI_AMD_CLIP_HOST_PREPROC"]
    assert torch.equal(emb_d, emb_h)


@pytest.mark.gpu
def test_grammar_mask_kernel_matches_torch():
    """grammar_mask (sampling.hip): rows with a slot get -inf outside that slot's allowed-token
    mask; rows with slot -1 are untouched."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    B, V, S = 6, 128256, 4
    lg = torch.randn(B, V, generator=g).to(dev)
    pool = (torch.rand(S, V, generator=g) < 0.1).to(dev)
    slot = torch.tensor([2, -1, 0, 3, -1, 2], dtype=torch.int32, device=dev)
    ref = lg.clone()
    for b in range(B):
        if int(slot[b]) >= 0:
            ref[b].masked_fill_(~pool[int(slot[b])], float("-inf"))
    out = lg.clone()
    ops.grammar_mask(out, slot, pool)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("T", [1, 2])
@pytest.mark.parametrize("fmts", [(GGMLType.Q4_K, GGMLType.Q6_K), (GGMLType.Q8_0, GGMLType.Q8_0)])
def test_moe_gemv_decode(T, fmts):
    """1-2 token MoE decode on the int8-dot GEMV (moe_gemv_kernel): device routing ids, SwiGLU +
    routing weight fused into the down prologue; vs the fp32 reference of the same weights.  A
    pair routed to another rank's expert (id >= E_local) contributes zero."""
    E, topk, D, F = 8, 2, 512, 768
    gu = [_qw(2 * F, D, fmts[0], seed=10 + e) for e in range(E)]
    dn = [_qw(D, F, fmts[1], seed=30 + e) for e in range(E)]
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    assert ops.moe_gemv_ok(mg, T) and ops.moe_gemv_ok(md, T)
    x = torch.randn(T, D, device=DEV).to(torch.bfloat16)
    ids = torch.stack([torch.randperm(E)[:topk] for _ in range(T)]).to(torch.int32).view(-1)
    if T == 2:
        ids[3] = E  # another rank's expert
    ids = ids.to(DEV)
    wts = torch.rand(T * topk, device=DEV)
    g = ops.moe_gemv(x, mg, ids, topk, T, E)
    z = ops.moe_gemv(None, md, ids, topk, T, E, act_src=g, act_mode=ops.ACT_SWIGLU, wts=wts).dense().cpu()
    xc, idc, wc = x.float().cpu(), ids.cpu().long(), wts.cpu()
    ref = torch.zeros(T, D)
    for p in range(T * topk):
        e = int(idc[p])
        if e >= E:
            continue
        h = xc[p // topk] @ gu[e].ref.t()
        a = torch.nn.functional.silu(h[:F]) * h[F:]
        ref[p // topk] += float(wc[p]) * (a @ dn[e].ref.t())
    err = float((z - ref).abs().max() / ref.abs().max())
    assert err < 3e-2, err


@pytest.mark.parametrize("cls_token", [True, False])
@pytest.mark.parametrize("heads", [2, 4])
def test_clip_tower_native_ops_match_fp32(tmp_path, cls_token, heads):
    """The vision tower on the native ops (ops.linear projections, fused residual + LayerNorm in
    add_norm, act-kernel GELU; 64-wide heads: non-causal MFMA attention, ops.attn_dense) vs the
    fp32 PyTorch tower on the CPU, same mmproj and pixels: every projected patch embedding row
    close in cosine and relative L2."""
    from localai_amd.models import synth
    from localai_amd.models.clip import ClipVision
    kw = dict(out_dim=256, dim=128, n_layer=2, heads=heads, ffn=256, image_size=56, patch=14)
    if not cls_token:
        kw["siglip"] = True
    mm = synth.write_mmproj(str(tmp_path / "mm.gguf"), **kw)
    gpu, cpu = ClipVision(mm, DEV), ClipVision(mm, torch.device("cpu"), dtype=torch.float32)
    assert gpu.native and not cpu.native
    pix = torch.randn(3, 3, 56, 56)
    a = gpu.encode_tiles(pix.to(DEV)).float().cpu()
    b = cpu.encode_tiles(pix)
    assert a.shape == b.shape
    cos = torch.nn.functional.cosine_similarity(a.reshape(-1, a.shape[-1]), b.reshape(-1, b.shape[-1]), dim=1)
    rel = float((a - b).norm() / b.norm())
    assert float(cos.min()) > 0.995 and rel < 5e-2, (float(cos.min()), rel)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("C", [4096, 1000, 7])
def test_gather_rows_kernel(dtype, C):
    """gather_rows_kernel (16-byte and byte-wise rows) vs torch indexing, fill rows for -1."""
    src = torch.randn(50, C, device=DEV).to(dtype)
    fill = torch.randn(C, device=DEV).to(dtype)
    idx = torch.tensor([3, -1, 49, 0, 0, -1, 17], dtype=torch.long, device=DEV)
    got = ops.gather_rows(src, idx, fill)
    ref = src[idx.clamp(min=0)].clone()
    ref[idx < 0] = fill
    assert torch.equal(got, ref)


def test_gemv_dp4_wide_batch1_variant():
    """Batch-1 GEMVs with N >= 16384 launch with four 8-row slots per wave (per-call variant 9):
    numerics vs fp32, repeated launches bit-identical, M=2 (variant 5) agreeing per row."""
    N, K = 16400, 1024
    w = _qw(N, K, GGMLType.Q4_K, seed=41)
    x = torch.randn(2, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    y1 = ops.linear(x[:1], w, force="dp4").dense()
    assert (y1.cpu() - ref[:1]).abs().max().item() < tol
    assert torch.equal(y1, ops.linear(x[:1], w, force="dp4").dense())
    y2 = ops.linear(x, w, force="dp4").dense().cpu()
    assert (y2 - ref).abs().max().item() < tol


@pytest.mark.parametrize("n,L,H,Dh", [(3, 577, 16, 64), (2, 50, 12, 64), (1, 130, 4, 128), (2, 33, 5, 80)])
def test_attn_dense_noncausal(n, L, H, Dh):
    """Vision-tower self-attention on the MFMA flash kernel (la_attn_dense: non-causal, q|k|v read
    in place from the fused projection output) vs the fp32 PyTorch softmax attention; ragged L
    (not a multiple of the 64-row query tile or the 32-key tile)."""
    D = H * Dh
    qkv = (torch.randn(n * L, 3 * D, device=DEV) * 0.5).to(torch.bfloat16)
    out = ops.attn_dense(qkv, n, L, H)
    torch.cuda.synchronize()
    q, k, v = qkv.float().cpu().view(n, L, 3, H, Dh).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) * Dh ** -0.5, -1) @ v).transpose(1, 2).reshape(n * L, D)
    got = out.float().cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.9999, cos


@pytest.mark.parametrize("T,E,topk,mode,renorm,ep", [(1, 8, 2, 0, True, False), (2, 8, 2, 0, True, True),
                                                      (37, 60, 4, 0, False, False), (5, 16, 2, 1, True, False)])
def test_add_norm_router_matches_unfused(T, E, topk, mode, renorm, ep):
    """add_norm_router (one launch) == add_norm + moe_router: identical bf16 rows and residual,
    identical expert ids, routing weights to fp32 rounding (block-order sums of the logits); and
    both against the plain fp32 PyTorch oracle of the same op (residual add, RMS / layer norm,
    softmax router on the bf16 row, top-k, renormalisation, local expert ids under EP)."""
    g = torch.Generator(device="cpu").manual_seed(T * 100 + E)
    D = 4096
    res0 = torch.randn(T, D, generator=g).to(DEV)
    slabs = torch.randn(3, T, D, generator=g).to(DEV) * 0.5
    w = (1.0 + 0.1 * torch.randn(D, generator=g)).to(DEV)
    b = (0.1 * torch.randn(D, generator=g)).to(DEV) if mode == 1 else None
    router = (torch.randn(E, D, generator=g) * 0.05).to(DEV)
    base, local = (E // 2, E // 2) if ep else (0, 0)
    ra, rb = res0.clone(), res0.clone()
    xa = ops.add_norm(ra, ops.Partial(slabs), w, b, 1e-5, mode)
    ida, wa = ops.moe_router(xa, router, topk, renorm, 1.0, base, local)
    fused = ops.add_norm_router(rb, ops.Partial(slabs), w, b, 1e-5, mode, router, topk, renorm, 1.0, base, local)
    assert fused is not None
    xb, idb, wb = fused
    torch.cuda.synchronize()
    assert torch.equal(ra, rb) and torch.equal(xa, xb)
    assert torch.equal(ida, idb)
    assert torch.allclose(wa, wb, rtol=1e-5, atol=1e-6)
    # fp32 oracle
    h = res0.cpu() + slabs.cpu().sum(0)
    if mode == 0:
        xn = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-5) * w.cpu()
    else:
        mu = h.mean(-1, keepdim=True)
        xn = (h - mu) * torch.rsqrt((h - mu).pow(2).mean(-1, keepdim=True) + 1e-5) * w.cpu() + b.cpu()
    assert torch.allclose(rb.cpu(), h, rtol=1e-6, atol=1e-5)
    assert (xb.float().cpu() - xn).abs().max().item() <= 1e-2 * xn.abs().max().item()
    p = torch.softmax(xb.float().cpu() @ router.cpu().t(), -1)
    pw, pidx = torch.topk(p, topk, -1)
    if renorm:
        pw = pw / pw.sum(-1, keepdim=True)
    local = (E // 2) if ep else E
    loc = pidx - base
    pids = torch.where((loc >= 0) & (loc < local), loc, torch.full_like(loc, local))
    # ids: equal wherever the k-th and (k+1)-th probabilities are not within fp32 rounding
    ps = torch.sort(p, -1, descending=True).values
    clear = (ps[:, topk - 1] - ps[:, topk]) > 1e-6 if topk < E else torch.ones(T, dtype=torch.bool)
    assert torch.equal(idb.cpu().long()[clear].sort(-1).values, pids[clear].sort(-1).values)
    got_w = wb.cpu().view(T, topk)
    for t in torch.nonzero(clear).flatten().tolist():
        ow = dict(zip(pidx[t].tolist(), pw[t].tolist()))
        gw = dict(zip((idb[t].cpu().long() + (base if ep else 0)).tolist(), got_w[t].tolist()))
        if ep:   # other ranks' experts share the id `local`: compare this rank's only
            ow = {k: v for k, v in ow.items() if base <= k < base + local}
            gw = {k: v for k, v in gw.items() if base <= k < base + local}
        assert ow.keys() == gw.keys()
        for k in ow:
            assert abs(ow[k] - gw[k]) <= 1e-5 + 1e-4 * abs(ow[k]), (t, k, ow[k], gw[k])
