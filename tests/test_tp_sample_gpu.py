"""Distributed sampler over vocabulary shards (TPInfo.sample_cols, sampling.hip tp_* kernels)
against the single-device sampler on the full rows: LocalAI's default chain (temperature 0.9,
top-k 40, top-p 0.95), min-p / typical / tail-free after top-k, greedy rows, repeat penalties on the
shards, and mirostat 2 with its mu update.  The ranks are simulated in one process: each shard runs
the kernels, and the exchange is the sum of the ranks' slots (what the custom all-reduce computes)."""
import numpy as np
import pytest
import torch

from localai_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _sim_sample(logits, prm, mu0, world, mirostat=True):
    B, V = logits.shape
    Vs = V // world
    prm_dev = torch.from_numpy(prm.view(np.uint8).copy()).to(DEV)
    C = ops.TP_SAMPLE_C
    cand = torch.zeros(world, B, C, 2, device=DEV)
    for r in range(world):
        ops.tp_topc(logits[:, r * Vs:(r + 1) * Vs].contiguous(), C, r * Vs, cand[r])
    vals = cand[..., 0].permute(1, 0, 2).contiguous().view(B, world * C)
    ids = cand[..., 1].permute(1, 0, 2).contiguous().view(B, world * C)
    idx = ops.sample(vals, prm, mu=torch.zeros(B, device=DEV), params_dev=prm_dev)
    out = ids.gather(1, idx.long().unsqueeze(1)).squeeze(1).to(torch.int32)
    mus = [mu0.clone() for _ in range(world)]
    if mirostat:
        shards = [logits[:, r * Vs:(r + 1) * Vs].contiguous() for r in range(world)]
        x1, x2, x3 = torch.zeros(world, B, 3, device=DEV), torch.zeros(world, B, device=DEV), \
            torch.zeros(world, B, 2, device=DEV)
        for phase, buf in ((1, x1), (2, x2), (3, x3)):
            parts = [torch.zeros_like(buf) for _ in range(world)]
            for r in range(world):
                ops.tp_mirostat(phase, shards[r], r * Vs, world, r, prm_dev, mus[r], x1, x2, x3, parts[r][r], None)
            buf.copy_(sum(parts))
        outs = [out.clone() for _ in range(world)]
        for r in range(world):
            ops.tp_mirostat(4, shards[r], r * Vs, world, r, prm_dev, mus[r], x1, x2, x3, None, outs[r])
        for r in range(1, world):   # every rank ends with the same tokens and mu
            assert torch.equal(outs[r], outs[0])
            assert torch.equal(mus[r], mus[0])
        out = outs[0]
    return out, mus[0]


def _params(B, **kw):
    prm = np.zeros(B, dtype=ops.SAMPLE_ROW_DTYPE)
    prm["temp"], prm["top_p"], prm["min_p"], prm["typical_p"], prm["tfs_z"] = 0.9, 0.95, 0.05, 1.0, 1.0
    prm["top_k"], prm["tau"], prm["eta"] = 40, 5.0, 0.1
    for k, v in kw.items():
        prm[k] = v
    prm["seed"] = np.arange(B) * 7919 + 11
    prm["counter"] = np.arange(B) % 5
    return prm


def _logits(B, V, seed, scale=3.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(B, V, device=DEV, generator=g) * scale


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("chain", ["default", "typical_tfs", "greedy", "topk1", "topk64"])
def test_tp_standard_chain_matches_full_row(world, chain):
    B, V = 64, 128256 // 8 * 8
    kw = {"default": {}, "typical_tfs": {"typical_p": 0.9, "tfs_z": 0.95}, "greedy": {"temp": 0.0},
          "topk1": {"top_k": 1}, "topk64": {"top_k": 64, "top_p": 1.0, "min_p": 0.0}}[chain]
    prm = _params(B, **kw)
    lg = _logits(B, V, seed=world * 31 + len(chain))
    ref = ops.sample(lg, prm, mu=torch.zeros(B, device=DEV))
    got, _ = _sim_sample(lg, prm, torch.zeros(B, device=DEV), world, mirostat=False)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref.cpu()), (got.cpu()[:8], ref.cpu()[:8])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_mirostat2_matches_full_row(world):
    """Mirostat 2: the same token for (almost) every row and the same mu update; the distributed
    sums differ from the full-row block sum only in rounding, so a draw landing within an ulp of a
    boundary may pick the neighbour -- at most one row in 64 here."""
    B, V = 64, 32000
    prm = _params(B, mirostat=2, temp=1.0)
    mu0 = torch.full((B,), 10.0, device=DEV)
    for scale in (1.0, 4.0, 8.0):
        lg = _logits(B, V, seed=world * 7 + int(scale), scale=scale)
        mu_ref = mu0.clone()
        ref = ops.sample(lg, prm, mu=mu_ref)
        got, mu_got = _sim_sample(lg, prm, mu0.clone(), world)
        torch.cuda.synchronize()
        same = (got.cpu() == ref.cpu())
        assert int(same.sum()) >= B - 1, (scale, int(same.sum()))
        assert torch.allclose(mu_got.cpu()[same], mu_ref.cpu()[same], rtol=1e-4, atol=1e-4)


def test_tp_penalties_on_shards():
    """Repeat / frequency / presence penalties applied to each shard's own columns equal the
    full-row penalties."""
    B, V, world = 8, 4096, 4
    Vs = V // world
    lg = _logits(B, V, seed=3)
    hist = torch.randint(0, V, (B, 32), dtype=torch.int32, device=DEV)
    hl = torch.full((B,), 32, dtype=torch.int32, device=DEV)
    pen = torch.tensor([[1.3, 0.2, 0.4]] * B, device=DEV)
    ref = ops.penalties(lg.clone(), hist, hl, pen)
    shards = [lg[:, r * Vs:(r + 1) * Vs].contiguous() for r in range(world)]
    for r in range(world):
        ops.penalties(shards[r], hist, hl, pen, col0=r * Vs)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(shards, 1).cpu(), ref.cpu())
