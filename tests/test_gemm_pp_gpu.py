"""Prefill GEMM (ops/csrc/gemm_pp.hip) against the plain fp32 PyTorch reference: every weight
format it takes, ragged M / N (off the 256 x 256 tile), split-K slabs, the two-weight launch
(q|k beside v) and the fused gate|up + SwiGLU / GeGLU epilogue."""
import numpy as np
import pytest
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, quantize

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
FMTS = [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.F16]


def _qw(N, K, t, seed=0, std=0.05):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((N, K)).astype(np.float32) * std
    return ops.QWeight.from_raw(quantize(w, t), t, (N, K), DEV, keep_ref=True)


def _check(y, ref, tol=2e-2):
    y = y.float().cpu()
    assert torch.isfinite(y).all()
    err = (y - ref).abs().max().item()
    assert err < tol * max(1.0, ref.abs().max().item()), err
    cos = torch.nn.functional.cosine_similarity(y.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.9999, cos


@pytest.mark.parametrize("t", FMTS)
@pytest.mark.parametrize("M,N,K", [(300, 272, 1024), (1000, 1040, 512), (256, 256, 2048)])
def test_pp_formats_ragged(t, M, N, K):
    w = _qw(N, K, t, seed=M + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    assert ops.pp_ok([w], K, 1)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_pp(x, [w], 1, out, N)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("S", [2, 4])
def test_pp_splits(t, S):
    M, N, K = 520, 528, 2048
    w = _qw(N, K, t, seed=S)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    assert ops.pp_ok([w], K, S)
    out = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=DEV)
    ops._run_pp(x, [w], S, out, N)
    torch.cuda.synchronize()
    _check(out.sum(0), ref)


def test_pp_two_weights():
    """q|k (Q4_K) beside v (Q6_K) in one launch, as the fused q|k|v projection runs."""
    M, K = 700, 1024
    wa = _qw(640, K, GGMLType.Q4_K, seed=1)
    wb = _qw(128, K, GGMLType.Q6_K, seed=2)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = torch.cat([x.float().cpu() @ wa.ref.t(), x.float().cpu() @ wb.ref.t()], 1)
    out = torch.full((M, 768), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_pp(x, [wa, wb], 1, out, 768)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("mode", [ops.ACT_SWIGLU, ops.ACT_GEGLU])
def test_pp_glu(t, mode):
    M, F, K = 600, 400, 1024
    w = _qw(2 * F, K, t, seed=7)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = x.float().cpu() @ w.ref.t()
    g, u = y[:, :F], y[:, F:]
    act = torch.nn.functional.silu(g) if mode == ops.ACT_SWIGLU else torch.nn.functional.gelu(g, approximate="tanh")
    ref = act * u
    out = torch.full((M, F), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_pp_glu(x, (w, 0, w, F), F, mode, out)
    torch.cuda.synchronize()
    _check(out, ref, 3e-2)


def test_pp_deterministic_and_no_oob():
    """Same bits on every launch; rows past M / columns past N are never written."""
    M, N, K = 260, 260, 1024
    w = _qw(N, K, GGMLType.Q4_K, seed=11)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    big = torch.full((M + 8, N + 8), 7.0, dtype=torch.bfloat16, device=DEV)
    view = big[:M]
    outs = []
    for _ in range(3):
        o = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops._run_pp(x, [w], 1, o, N)
        outs.append(o)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    rc = ops.lib().la_gemm_pp(w.fmt, *w.tile_planes(), N, K, x.data_ptr(), K, M, 1, view.data_ptr(), N + 8, 0, 1,
                              ops._stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert (big[:, N:] == 7.0).all() and (big[M:] == 7.0).all()
    _check(view[:, :N], x.float().cpu() @ w.ref.t())
