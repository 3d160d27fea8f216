"""Quantised tile GEMM (ops/csrc/gemm_q.hip) against the plain fp32 PyTorch reference:
every tile shape, every weight format, split-K, bf16 output, ragged M / N, and the
Llama-3-8B production shapes at decode batch 256 through the engine's dispatch."""
import numpy as np
import pytest
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, quantize

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
FMTS = [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.F16]


def _qw(N, K, t, seed=0, std=0.05):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((N, K)).astype(np.float32) * std
    return ops.QWeight.from_raw(quantize(w, t), t, (N, K), DEV, keep_ref=True)


def _run(w, x, tile, S, bf16=False):
    M, K = x.shape
    N = w.N
    p0, p1, g = w.tile_planes()
    if bf16:
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        slab = 0
    else:
        out = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=DEV)
        slab = M * N
    rc = ops.lib().la_qgemm_tile(w.fmt, p0, p1, g, N, K, x.data_ptr(), K, M, S, out.data_ptr(), N, slab, int(bf16),
                                 tile, 0, ops._stream())
    assert rc == 0, rc
    torch.cuda.synchronize()
    return out.float().cpu() if bf16 else out.sum(0).cpu()


def _check(y, ref, tol=2e-2):
    assert torch.isfinite(y).all()
    err = (y - ref).abs().max().item()
    assert err < tol * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("t", FMTS)
@pytest.mark.parametrize("tile", sorted(ops.GQ_TILES))
def test_tile_gemm_formats(t, tile):
    """N off every tile width, M off every tile height, K = 6 super-blocks."""
    N, K, M = 200, 1536, 150
    w = _qw(N, K, t, seed=tile)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    _check(_run(w, x, tile, 1), ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
def test_tile_gemm_splits(t):
    """split-K at odd K-step boundaries (the Q6_K K-step permutation spans 4 K-steps)."""
    N, K, M = 130, 3584, 256
    w = _qw(N, K, t, seed=3)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    for tile in (0, 1, 4, 6):
        for S in (1, 3, 5, 8, 14):
            _check(_run(w, x, tile, S), ref, 3e-2)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.F16])
def test_tile_gemm_bf16_out_large_m(t):
    N, K, M = 384, 1024, 1100
    w = _qw(N, K, t, seed=5)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    _check(_run(w, x, 0, 1, bf16=True), ref)


def test_tile_gemm_deterministic():
    w = _qw(512, 2048, GGMLType.Q4_K, seed=9)
    x = torch.randn(256, 2048, device=DEV).to(torch.bfloat16)
    a = _run(w, x, 0, 2)
    b = _run(w, x, 0, 2)
    assert torch.equal(a, b)


def test_tile_gemm_asymmetric_identity():
    """A = I (rows of the identity) with an asymmetric W: the output must be W^T exactly as
    dequantised (catches a transposed C write / swapped fragment maps)."""
    N, K = 64, 256
    w = _qw(N, K, GGMLType.Q8_0, seed=2)
    x = torch.zeros(K, K, dtype=torch.bfloat16, device=DEV)
    x[torch.arange(K), torch.arange(K)] = 1
    y = _run(w, x, 3, 1)
    ref = w.ref.t().to(torch.bfloat16).float()
    assert (y - ref).abs().max().item() < 1e-6


@pytest.mark.parametrize("M", [96, 160, 256])
def test_linear_dispatch_llama3_shapes(M):
    """The engine's dispatch (autotuned tile choice) at decode batch sizes on the Llama-3-8B
    projection shapes (q|k|v mixed Q4_K + Q6_K, o, gate|up, down) against fp32."""
    K = 4096
    shapes = {
        "qkv": ([(4096, GGMLType.Q4_K), (1024, GGMLType.Q4_K), (1024, GGMLType.Q6_K)], K),
        "o": ([(4096, GGMLType.Q4_K)], K),
        "gate_up": ([(14336, GGMLType.Q4_K), (14336, GGMLType.Q4_K)], K),
        "down": ([(4096, GGMLType.Q6_K)], 14336),
    }
    x_full = torch.randn(M, 14336, device=DEV).to(torch.bfloat16)
    for name, (parts, k) in shapes.items():
        ws = [_qw(n, k, t, seed=i) for i, (n, t) in enumerate(parts)]
        x = x_full[:, :k].contiguous()
        y = ops.linear_multi(x, ws).dense().cpu()
        ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
        rel = ((y - ref).norm() / ref.norm()).item()
        cos = torch.nn.functional.cosine_similarity(y.flatten(), ref.flatten(), dim=0).item()
        assert rel < 1e-2 and cos > 0.9999, (name, rel, cos)
        assert ops._GEMM_CHOICE, "autotune recorded no choice"
        for key, ch in ops._GEMM_CHOICE.items():
            assert ch[0] in ("tile", "q32", "bs"), (key, ch)


@pytest.mark.parametrize("tile", [7, 8, 12])
@pytest.mark.parametrize("S", [1, 3])
def test_tile_gemm_two_segments_one_launch(tile, S):
    """Q4_K q|k beside a Q6_K v (and the reverse) in one la_qgemm_tile2 launch."""
    K, M = 1536, 200
    for fa, fb in ((GGMLType.Q4_K, GGMLType.Q6_K), (GGMLType.Q6_K, GGMLType.Q4_K)):
        ws = [_qw(320, K, fa, seed=1), _qw(96, K, fb, seed=2)]
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        Ntot = 416
        out = (torch.full((M, Ntot), float("nan"), dtype=torch.bfloat16, device=DEV) if S == 1 else
               torch.full((S, M, Ntot), float("nan"), dtype=torch.float32, device=DEV))
        ops._run_tile(x, ws, S, out, Ntot, tile)
        torch.cuda.synchronize()
        y = out.float().cpu() if S == 1 else out.sum(0).cpu()
        ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
        _check(y, ref)


@pytest.mark.parametrize("t", FMTS)
@pytest.mark.parametrize("tile", [6, 7, 8, 12, 14])
def test_glu_fused_gate_up(t, tile):
    """gate|up with SwiGLU / GeGLU in the tile epilogue (la_qgemm_glu) vs fp32: two weights, and
    the halves of one fused [2F, K] weight; F off every half-tile width, ragged M."""
    F, K, M = 200, 768, 150
    g, u = _qw(F, K, t, seed=40 + tile), _qw(F, K, t, seed=41 + tile)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    xc = x.float().cpu()
    for mode in (ops.ACT_SWIGLU, ops.ACT_GEGLU):
        gr, ur = xc @ g.ref.t(), xc @ u.ref.t()
        act = (torch.nn.functional.silu(gr) if mode == ops.ACT_SWIGLU
               else torch.nn.functional.gelu(gr, approximate="tanh"))
        ref = act * ur
        out = torch.full((M, F), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops._run_glu(x, (g, 0, u, 0), F, mode, tile, out)
        torch.cuda.synchronize()
        _check(out.float().cpu(), ref, 3e-2)
    # one [2F, K] weight (Phi-3 style fused gate_up): up rows start at F (F % 16 == 0)
    F2 = 208
    w = _qw(2 * F2, K, t, seed=50 + tile)
    out = torch.full((M, F2), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_glu(x, (w, 0, w, F2), F2, ops.ACT_SWIGLU, tile, out)
    torch.cuda.synchronize()
    full = xc @ w.ref.t()
    _check(out.float().cpu(), torch.nn.functional.silu(full[:, :F2]) * full[:, F2:], 3e-2)


def test_glu_linear_dispatch():
    """ops.glu_linear (autotuned fused vs unfused) returns act(gate) * up at a decode batch."""
    F, K, M = 1024, 1024, 200
    ws = [_qw(F, K, GGMLType.Q4_K, seed=61), _qw(F, K, GGMLType.Q4_K, seed=62)]
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    h = ops.glu_linear(x, ws, F, ops.ACT_SWIGLU)
    if h is None:  # unfused won the autotune: the decoder then runs GEMM + act
        h = ops.act(ops.linear_multi(x, ws), F, ops.ACT_SWIGLU)
    xc = x.float().cpu()
    ref = torch.nn.functional.silu(xc @ ws[0].ref.t()) * (xc @ ws[1].ref.t())
    _check(h.float().cpu(), ref, 3e-2)


# ---------------------------------------------------------------- gemm_q32.hip (32x32x16 MFMA)
Q32_VARS = sorted(ops.Q32_TILES)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("var", Q32_VARS)
def test_q32_formats(t, var):
    """Every variant (tile shape, 4 or 8 waves, schedule) and format vs fp32: N off every tile
    width, M off every tile height, split-K over odd K-step boundaries, bf16 output."""
    N, K, M = 200, 1536, 150
    w = _qw(N, K, t, seed=100 + var)
    if not ops.q32_ok([w], var):
        pytest.skip("variant not built for this format")
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    for S in (1, 5):
        out = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=DEV)
        ops._run_q32(x, [w], S, out, N, var)
        torch.cuda.synchronize()
        _check(out.sum(0).cpu(), ref)
    ob = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_q32(x, [w], 1, ob, N, var)
    torch.cuda.synchronize()
    _check(ob.float().cpu(), ref)


def test_q32_asymmetric_identity():
    """A = I with an asymmetric W: the output is W^T exactly as dequantised (swapped fragment
    maps or a transposed C write would show)."""
    N, K = 96, 256
    w = _qw(N, K, GGMLType.Q8_0, seed=3)
    x = torch.zeros(K, K, dtype=torch.bfloat16, device=DEV)
    x[torch.arange(K), torch.arange(K)] = 1
    for var in (0, 8):
        out = torch.full((1, K, N), float("nan"), dtype=torch.float32, device=DEV)
        ops._run_q32(x, [w], 1, out, N, var)
        torch.cuda.synchronize()
        ref = w.ref.t().to(torch.bfloat16).float()
        assert (out[0].cpu() - ref).abs().max().item() < 1e-6


@pytest.mark.parametrize("var", [0, 1, 3, 4, 8, 9])
def test_q32_two_segments_one_launch(var):
    """Q4_K q|k beside a Q6_K v (and the reverse) in one la_qgemm32_2 launch."""
    K, M = 1536, 200
    for fa, fb in ((GGMLType.Q4_K, GGMLType.Q6_K), (GGMLType.Q6_K, GGMLType.Q4_K)):
        ws = [_qw(320, K, fa, seed=11), _qw(96, K, fb, seed=12)]
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        Ntot = 416
        for S in (1, 3):
            out = torch.full((S, M, Ntot), float("nan"), dtype=torch.float32, device=DEV)
            ops._run_q32(x, ws, S, out, Ntot, var)
            torch.cuda.synchronize()
            ref = torch.cat([x.float().cpu() @ w.ref.t() for w in ws], -1)
            _check(out.sum(0).cpu(), ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("var", [0, 1, 2, 4, 5, 7, 8, 9])
def test_q32_glu(t, var):
    """gate|up with SwiGLU / GeGLU in the q32 epilogue vs fp32 (two weights, and the halves of
    one fused [2F, K] weight)."""
    F, K, M = 200, 768, 150
    g, u = _qw(F, K, t, seed=70 + var), _qw(F, K, t, seed=71 + var)
    if not ops.q32_ok([g], var):
        pytest.skip("variant not built for this format")
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    xc = x.float().cpu()
    for mode in (ops.ACT_SWIGLU, ops.ACT_GEGLU):
        gr, ur = xc @ g.ref.t(), xc @ u.ref.t()
        act = (torch.nn.functional.silu(gr) if mode == ops.ACT_SWIGLU
               else torch.nn.functional.gelu(gr, approximate="tanh"))
        out = torch.full((M, F), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops._run_glu(x, (g, 0, u, 0), F, mode, 100 + var, out)
        torch.cuda.synchronize()
        _check(out.float().cpu(), act * ur, 3e-2)
    F2 = 208
    w = _qw(2 * F2, K, t, seed=80 + var)
    out = torch.full((M, F2), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_glu(x, (w, 0, w, F2), F2, ops.ACT_SWIGLU, 100 + var, out)
    torch.cuda.synchronize()
    full = xc @ w.ref.t()
    _check(out.float().cpu(), torch.nn.functional.silu(full[:, :F2]) * full[:, F2:], 3e-2)
