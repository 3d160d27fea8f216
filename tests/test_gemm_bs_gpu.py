"""Shared-dequant-image GEMM (ops/csrc/gemm_bs.hip) against the plain fp32 PyTorch reference:
every weight format (Q4_K, Q6_K, Q8_0, bf16), every tile variant, ragged M / N (off the tile),
split-K slabs, the two-weight q|k + v launch and the fused gate|up GLU epilogue."""
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


def _check(y, ref, tol=2e-2):
    y = y.float().cpu()
    assert torch.isfinite(y).all()
    err = (y - ref).abs().max().item()
    assert err < tol * max(1.0, ref.abs().max().item()), err
    cos = torch.nn.functional.cosine_similarity(y.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.9999, cos


@pytest.mark.parametrize("t", FMTS)
@pytest.mark.parametrize("var", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(77, 260, 512), (256, 384, 1024), (300, 1000, 768)])
def test_bs_formats_ragged(t, var, M, N, K):
    w = _qw(N, K, t, seed=M + N + var)
    assert ops.bs_ok([w])
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_bs(x, [w], 1, out, N, var)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("S", [2, 3, 8])
def test_bs_splits(t, S):
    """fp32 split-K slabs, including splits that own one or two K-steps (the ring's tail paths)."""
    M, N, K = 256, 512, 1024
    w = _qw(N, K, t, seed=S)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    out = torch.full((S, M, N), float("nan"), dtype=torch.float32, device=DEV)
    ops._run_bs(x, [w], S, out, N, 0)
    torch.cuda.synchronize()
    _check(out.sum(0), ref)


@pytest.mark.parametrize("var", [0, 1])
def test_bs_two_weights(var):
    """q|k (Q4_K) beside v (Q6_K) in one launch, as the fused q|k|v projection runs."""
    M, K = 200, 1024
    wa = _qw(640, K, GGMLType.Q4_K, seed=1)
    wb = _qw(128, K, GGMLType.Q6_K, seed=2)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = torch.cat([x.float().cpu() @ wa.ref.t(), x.float().cpu() @ wb.ref.t()], 1)
    out = torch.full((2, M, 768), float("nan"), dtype=torch.float32, device=DEV)
    ops._run_bs(x, [wa, wb], 2, out, 768, var)
    torch.cuda.synchronize()
    _check(out.sum(0), ref)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
@pytest.mark.parametrize("mode", [ops.ACT_SWIGLU, ops.ACT_GEGLU])
@pytest.mark.parametrize("var", [0, 2])
def test_bs_glu(t, mode, var):
    M, F, K = 230, 400, 1024
    w = _qw(2 * F, K, t, seed=7)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    y = x.float().cpu() @ w.ref.t()
    g, u = y[:, :F], y[:, F:]
    act = torch.nn.functional.silu(g) if mode == ops.ACT_SWIGLU else torch.nn.functional.gelu(g, approximate="tanh")
    ref = act * u
    out = torch.full((M, F), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops._run_bs_glu(x, (w, 0, w, F), F, mode, var, out)
    torch.cuda.synchronize()
    _check(out, ref)


def test_bs_large_prefill_shape():
    """A prefill-sized chunk (M = 2048) on the 256 x 256 tile, Q4_K, bf16 output."""
    M, N, K = 2048, 1536, 2048
    w = _qw(N, K, GGMLType.Q4_K, seed=11)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    ref = x.float().cpu() @ w.ref.t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops._run_bs(x, [w], 1, out, N, 2)
    torch.cuda.synchronize()
    _check(out, ref)
