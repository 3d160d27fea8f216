"""Grouped MoE GEMMs on the shared-dequant-image tile (gemm_bs.hip bsmoe_kernel via ops.moe_glu_bs /
ops.moe_down_bs) vs fp32 PyTorch references of the same quantised experts: every tile variant,
balanced and skewed routing (one expert with many 256-row chunks, experts with none), Q4_K / Q6_K /
Q8_0, expert parallelism (pairs of other ranks' experts skipped), the decoder's MoE layer on a
prefill-sized chunk against the dense per-expert path it replaces, and a graph capture (the launch
reads the grouping on the device only)."""
import pytest
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType

from test_moe32_gpu import _check, _ref, _setup

pytestmark = pytest.mark.gpu


def _run(x, mg, md, order, off, topk, T, wts, var, zero=False):
    h = ops.moe_glu_bs(x, mg, order, off, topk, T, var=var)
    return h, ops.moe_down_bs(h, md, order, off, topk, T, wts, zero=zero, var=var)


@pytest.mark.parametrize("var", sorted(ops.BS_TILES))
@pytest.mark.parametrize("T,skew", [(37, False), (600, False), (300, True)])
def test_moe_bs_variants(var, T, skew):
    E, topk, D, F = 8, 2, 512, 768
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q6_K, skew, seed=5)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    h, d = _run(x, mg, md, order, off, topk, T, wts, var)
    hs, ref = _ref(gu, dn, x, ids, wts, topk, E)
    o, offc = order.cpu().tolist(), off.cpu().tolist()
    hc = h.float().cpu()
    for e in range(E):  # grouped row r holds pair order[r]
        for r in range(offc[e], offc[e + 1]):
            _check(hc[r], hs[o[r]])
    _check(d.dense(), ref)


@pytest.mark.parametrize("tg,td", [(GGMLType.Q8_0, GGMLType.Q4_K), (GGMLType.Q6_K, GGMLType.Q8_0)])
def test_moe_bs_formats(tg, td):
    E, topk, T, D, F = 4, 2, 300, 1024, 1024
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, tg, td, seed=13)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    _, ref = _ref(gu, dn, x, ids, wts, topk, E)
    _, d = _run(x, mg, md, order, off, topk, T, wts, 0)
    _check(d.dense(), ref)


def test_moe_bs_expert_parallel():
    """This rank holds experts 0..3 of 8: pairs routed to group El are skipped, their slab rows
    stay zero, and every local pair matches."""
    El, topk, T, D, F = 4, 2, 400, 512, 768
    gu, dn, x, ids, ids_d, wts = _setup(El, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q4_K, seed=23, ep_total=8)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, El + 1)
    _, d = _run(x, mg, md, order, off, topk, T, wts, 0, zero=True)
    _, ref = _ref(gu, dn, x, ids, wts, topk, El)
    _check(d.dense(), ref)


def test_moe_bs_graph_replay_new_routing():
    """One captured launch pair serves any routing: the grid is sized for the worst case and the
    kernel reads the grouping on the device, so replaying after re-routing in place matches."""
    E, topk, T, D, F = 8, 2, 512, 512, 768
    gu, dn, x, ids, ids_d, wts = _setup(E, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q4_K, seed=41)
    mg, md = ops.MoEWeights(gu), ops.MoEWeights(dn)
    order, off = ops.moe_route(ids_d, E)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _run(x, mg, md, order, off, topk, T, wts, 0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        _, d = _run(x, mg, md, order, off, topk, T, wts, 0)
    for skew in (True, False):
        _, _, _, ids2, ids2_d, _ = _setup(E, topk, T, D, F, GGMLType.Q4_K, GGMLType.Q4_K, skew, seed=43)
        o2, f2 = ops.moe_route(ids2_d, E)
        order.copy_(o2)
        off.copy_(f2)
        g.replay()
        torch.cuda.synchronize()
        _, ref = _ref(gu, dn, x, ids2, wts, topk, E)
        _check(d.dense(), ref)


def test_decoder_moe_prefill_bs_matches_dense(tmp_path, monkeypatch):
    """A Mixtral-shaped layer on a prefill-sized chunk: the grouped bs path (opt-in, one launch per
    projection, no host sync), the default grouped moe32 path below MOE_DENSE_MIN_T and the dense
    per-expert path agree."""
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.models import decoder, synth
    monkeypatch.setattr(ops, "MOE_BS", True)
    p = str(tmp_path / "mx.gguf")
    synth.write_model(p, "tiny-mixtral")
    eng = LLMEngine(EngineConfig(model_path=p, device="cuda:0", context_size=512, max_num_seqs=4,
                                 max_batched_tokens=2048))
    m = eng.model
    L = next(L for L in m.layers if L.experts is not None)
    if L.moe_gu is None or not ops.moe_bs_ok(L.moe_gu, L.moe_down, 1024):
        pytest.skip("synthetic Mixtral experts not on a bs format")
    T = 1024
    g = torch.Generator(device="cpu").manual_seed(7)
    xn = (torch.randn(T, m.hp.n_embd, generator=g) * 0.5).to(torch.bfloat16).to("cuda:0")
    calls = []
    orig = ops.moe_glu_bs
    monkeypatch.setattr(ops, "moe_glu_bs", lambda *a, **k: calls.append(1) or orig(*a, **k))
    a = ops.reduce(m._moe(L, xn)).float()
    assert calls, "the grouped bs path did not run"
    monkeypatch.setattr(ops, "MOE_BS", False)
    g32 = []
    orig32 = ops.moe_glu32
    monkeypatch.setattr(ops, "moe_glu32", lambda *a, **k: g32.append(1) or orig32(*a, **k))
    c = ops.reduce(m._moe(L, xn)).float()   # T < MOE_DENSE_MIN_T: grouped moe32
    assert g32, "the grouped moe32 path did not run"
    monkeypatch.setattr(decoder, "MOE_DENSE_MIN_T", 1)
    b = ops.reduce(m._moe(L, xn)).float()
    for got in (a, c):
        rel = ((got - b).norm() / b.norm()).item()
        assert rel < 1e-2, rel
