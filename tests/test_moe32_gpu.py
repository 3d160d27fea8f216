"""Grouped MoE GEMMs on the 32x32x16 tile (gemm_q32.hip moe32_kernel via ops.moe_glu32 /
ops.moe_down32) vs fp32 PyTorch references of the same quantised experts: every variant, balanced
and skewed routing (experts with several row chunks and experts with none), Q4_K / Q6_K / Q8_0,
split-K on the down projection, expert parallelism (pairs of other ranks' experts skipped), and
the decoder's MoE layer agreeing with the previous grouped path."""
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
    return ops.QWeight.from_raw(quantize(w, t), t, (N, K), DEV, keep_ref=True)


def _setup(E, topk, T, D, F, tg, td, skew=False, seed=0, ep_total=None):
    gu = [_qw(2 * F, D, tg, seed=seed + e) for e in range(E)]
    dn = [_qw(D, F, td, seed=seed + 100 + e) for e in range(E)]
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(T, D, generator=g).to(torch.bfloat16).to(DEV)
    tot = ep_total or E
    if skew:
        ids = torch.tensor([[0, 1]] * T, dtype=torch.int32)
    else:
        ids = torch.stack([torch.randperm(tot, generator=g)[:topk] for _ in range(T)]).to(torch.int32)
    ids_l = torch.where(ids < E, ids, torch.full_like(ids, E)) if ep_total else ids
    wts = torch.rand(T * topk, generator=g).to(DEV)
    return gu, dn, x, ids, ids_l.to(DEV), wts


def _ref(gu, dn, x, ids, wts, topk, E):
    """fp32: per pair h = silu(x Wg^T) * (x Wu^T) (rounded to bf16 as the kernel stores it), the
    weighted sum of h Wd^T over the token's picks."""
    xc = x.float().cpu()
    T = xc.shape[0]
    F = gu[0].N // 2
    out = torch.zeros(T, dn[0].N)
    hs = {}
    for p in range(T * topk):
        t, e = p // topk, int(ids.view(-1)[p])
        if e >= E:
            continue
        y = xc[t] @ gu[e].ref.t()
        h = (torch.nn.functional.silu(y[:F]) * y[F:]).to(torch.bfloat16).float()
        hs[p] = h
        out[t] += float(wts.view(-1)[p]) * (h @ dn[e].ref.t())
    return hs, out


def _check(got, ref, tol=2e-2):
    err = (got.float().cpu() - ref).abs().max().item()
    assert err < tol * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("var", sorted(ops.MOE32_TILES))
@pytest.mark.parametrize("T,skew", [(70, False), (256, False), (200, True)])
def test_moe32_variants(var, T, skew):
    E, topk, D, F = 8, 2, 512, 768
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q6_K, skew, seed=3)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    h = ops.moe_glu32(x, mg, order, off, topk, T, var=var)
    hs, ref = _ref(gu, dn, x, ids, wts, topk, E)
    o, offc = order.cpu().tolist(), off.cpu().tolist()
    hc = h.float().cpu()
    for e in range(E):  # grouped row r holds pair order[r]
        for r in range(offc[e], offc[e + 1]):
            _check(hc[r], hs[o[r]])
    d = ops.moe_down32(h, md, order, off, topk, T, wts, var=var)
    _check(d.dense(), ref)


@pytest.mark.parametrize("tg,td", [(GGMLType.Q8_0, GGMLType.Q4_K), (GGMLType.Q6_K, GGMLType.Q8_0)])
def test_moe32_formats_and_splits(tg, td, monkeypatch):
    E, topk, T, D, F = 4, 2, 96, 1024, 1024
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, tg, td, seed=11)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    _, ref = _ref(gu, dn, x, ids, wts, topk, E)
    h = ops.moe_glu32(x, mg, order, off, topk, T)
    for S in (1, 2, 4):
        monkeypatch.setattr(ops, "MOE32_SPLITS", S)
        d = ops.moe_down32(h, md, order, off, topk, T, wts)
        assert d.t.shape[0] == S * topk
        _check(d.dense(), ref)


def test_moe32_expert_parallel():
    """This rank holds experts 0..3 of 8: pairs routed to group El are skipped, their slab rows
    stay zero, and every local pair matches."""
    El, topk, T, D, F = 4, 2, 128, 512, 768
    gu, dn, x, ids, ids_d, wts = _setup(El, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q4_K, seed=21, ep_total=8)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, El + 1)
    h = ops.moe_glu32(x, mg, order, off, topk, T)
    d = ops.moe_down32(h, md, order, off, topk, T, wts, zero=True)
    _, ref = _ref(gu, dn, x, ids, wts, topk, El)
    _check(d.dense(), ref)


def test_moe32_matches_previous_grouped_path():
    """ops.moe_linear + act + moe_linear(down) (moe.hip) and moe_glu32 + moe_down32 agree."""
    E, topk, T, D, F = 8, 2, 160, 1024, 768
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q6_K, seed=31)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    g = ops.moe_linear(x, mg, order, off, topk, T)
    a = ops.moe_linear(ops.act(g, F, ops.ACT_SWIGLU), md, order, off, topk, T, down=True, wts=wts).dense()
    b = ops.moe_down32(ops.moe_glu32(x, mg, order, off, topk, T), md, order, off, topk, T, wts).dense()
    rel = ((a.float() - b.float()).norm() / a.float().norm()).item()
    assert rel < 1e-2, rel
