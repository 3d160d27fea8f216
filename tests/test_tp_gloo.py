"""Tensor parallelism over torch.distributed (gloo on CPU, world_size 2): the leader (rank 0)
takes requests and broadcasts them; the follower mirrors every step.  The greedy stream must be
identical on both ranks and match the unsharded model's first token (the RCCL path on MI355X
runs the same code with backend "nccl")."""
import os
import queue
import socket
import time

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q, ep=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
        from localai_amd.engine.sampling_params import SamplingParams
        from localai_amd.models.decoder import TPInfo
        ctrl = dist.new_group(backend="gloo")
        tp = TPInfo(rank=rank, world=world, group=dist.group.WORLD, ep=ep)
        eng = LLMEngine(EngineConfig(model_path=path, device="cpu", context_size=256, max_num_seqs=4,
                                     use_graphs=False), tp=tp, ctrl_group=ctrl)
        if rank == 0:
            outs = []
            for prompt in ("tensor parallel test", "second request"):
                res = eng.generate(prompt, SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True))
                outs.append((res["text"], res["completion_tokens"]))
            emb = eng.embed(["embed me"])[0]
            n_exp = len(eng.model.layers[0].experts or [])
            eng.shutdown()
            q.put((rank, outs, [float(v) for v in emb], n_exp))
        else:
            eng.run_follower()
            q.put((rank, eng.metrics["requests"], eng.metrics["gen_tokens"]))
    finally:
        dist.destroy_process_group()


import pytest


@pytest.fixture(params=["tiny-llama", "tiny-mixtral", "tiny-phi2", "tiny-qwen2moe", "tiny-gemma2", "tiny-phi3"])
def tp_model_path(request, tiny_model_path, tmp_path_factory):
    """Llama (dense GQA), Mixtral (TP-within-expert: every expert's F sharded, router replicated),
    Phi-2 (LayerNorm + biases, NEOX partial rotary, biases added once after the all-reduce) and
    Qwen2-MoE (unaligned expert F shards, sigmoid-gated shared expert sliced like a dense MLP),
    Gemma-2 (one kv head replicated on both ranks, post-norms on the reduced outputs, soft-capping)
    and Phi-3 (fused q|k|v and gate|up tensors sliced per rank)."""
    if request.param == "tiny-llama":
        return tiny_model_path
    from localai_amd.models import synth
    p = tmp_path_factory.mktemp("tp") / f"{request.param}.gguf"
    synth.write_model(str(p), request.param, exact=True)
    return str(p)


def test_tp2_leader_follower(tp_model_path):
    _run_tp2(tp_model_path)


def test_ep2_mixtral(tiny_model_path, tmp_path_factory):
    """Expert parallelism (TPInfo.ep): each rank holds half of the experts whole, the MoE output
    is summed by the all-reduce that closes the MLP; greedy output agrees with one rank."""
    from localai_amd.models import synth
    p = tmp_path_factory.mktemp("ep") / "tiny-mixtral.gguf"
    synth.write_model(str(p), "tiny-mixtral", exact=True)
    n_exp = _run_tp2(str(p), ep=True)
    from localai_amd.gguf import GGUFReader
    from localai_amd.models.hparams import HParams
    assert n_exp == HParams.from_gguf(GGUFReader(str(p))).n_expert // 2


def _run_tp2(tp_model_path, ep=False, world=2):
    tiny_model_path = tp_model_path
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    single = LLMEngine(EngineConfig(model_path=tiny_model_path, device="cpu", context_size=256, max_num_seqs=4,
                                    use_graphs=False))
    ref = single.generate("tensor parallel test", SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, tiny_model_path, q, ep)) for r in range(world)]
    for p in procs:
        p.start()
    out, t0 = {}, time.time()
    while len(out) < len(procs):
        try:
            r = q.get(timeout=2)
            out[r[0]] = r
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), "a TP rank crashed"
            assert time.time() - t0 < 300
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    _, outs, emb, n_exp = out[0]
    assert [n for _, n in outs] == [5, 5]
    for r in range(1, world):
        _, f_requests, f_tokens = out[r]
        assert f_requests == 2 and f_tokens == 10  # every follower ran the same two requests
    assert len(emb) == single.model.hp.n_embd
    # hidden states through every sharded layer (column/row-parallel GEMMs, the all-reduces, the
    # sharded attention / experts) against the unsharded model: numerically, not just the argmax
    import torch
    a, b = torch.tensor(emb), torch.tensor(single.embed(["embed me"])[0], dtype=torch.float32)
    rel = float((a - b).norm() / b.norm())
    cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
    assert rel < 2e-2 and cos > 0.9998, (rel, cos)
    # sharded reductions change bf16 summation order; the first token must agree
    assert outs[0][0][:1] == ref["text"][:1]
    return n_exp


def test_tp4_replicated_kv_heads(tiny_model_path):
    """TP=4 over a model with 2 kv heads: each kv head lives on the 2 ranks whose query heads read
    it (DecoderModel.kv_rep), so TP degrees above the kv-head count (Qwen2-7B at TP=8) work."""
    _run_tp2(tiny_model_path, world=4)


def test_tp2_chunked_row_parallel(tiny_model_path, monkeypatch):
    """Row-parallel outputs all-reduced chunk by chunk (the prefill overlap path: GEMM of chunk
    k+1 beside the all-reduce of chunk k on the comm stream) give the unsharded hidden states:
    forced on for every prefill of >= 2 rows, in 3 chunks."""
    monkeypatch.setenv("LOCALAI_AMD_TP_OVERLAP_ROWS", "2")
    monkeypatch.setenv("LOCALAI_AMD_TP_OVERLAP_CHUNKS", "3")
    _run_tp2(tiny_model_path)


def _logits_worker(rank, world, port, path, q):
    """One rank of a TP group: prefill a fixed sequence through the sharded model, then two decode
    steps; rank 0 reports every row of logits."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _sequence_logits(path, rank, world)))
    finally:
        dist.destroy_process_group()


def _sequence_logits(path, rank=0, world=1):
    import torch
    import torch.distributed as dist
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.models.decoder import ForwardBatch, TPInfo
    kw = {}
    if world > 1:
        kw = dict(tp=TPInfo(rank=rank, world=world, group=dist.group.WORLD), ctrl_group=dist.new_group(backend="gloo"))
    eng = LLMEngine(EngineConfig(model_path=path, device="cpu", context_size=128, max_num_seqs=2, use_graphs=False,
                                 block_size=16), **kw)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    toks = [17, 923, 41, 5000, 7, 7, 311, 28000, 95, 1024, 3, 64]
    T = len(toks)
    bt = i32([list(range(8))])
    fb = ForwardBatch(tokens=i32(toks), pos=i32(list(range(T))), slots=i32(list(range(T))), decode=False,
                      block_tables=bt, cu_q=i32([0, T]), ctx_lens=i32([T]))
    rows = [eng.model.forward(fb, eng.kv).float()]
    nxt = int(rows[-1][-1].argmax())
    for step in range(2):
        p = T + step
        fb = ForwardBatch(tokens=i32([nxt]), pos=i32([p]), slots=i32([p]), decode=True, block_tables=bt,
                          seq_lens=i32([p + 1]), max_len=p + 1)
        rows.append(eng.model.forward(fb, eng.kv).float())
        nxt = int(rows[-1][-1].argmax())
    return torch.cat(rows).tolist()


def test_tp8_per_token_logits_70b_shaped(tmp_path_factory):
    """TP=8 on a Llama-3-70B-shaped tiny model (8 kv heads: ONE kv head per rank, 8:1 GQA): every
    row of logits -- a 12-token prefill and two decode steps -- against the unsharded model
    (rel <= 1e-2, cosine >= 0.9999), not just the first token."""
    import torch
    from localai_amd.models import synth
    p = tmp_path_factory.mktemp("tp8") / "tiny-70b-shape.gguf"
    synth.write_model(str(p), "tiny-llama", exact=True, n_embd=512, n_head=16, n_head_kv=8, n_ff=1024)
    ref = torch.tensor(_sequence_logits(str(p)))
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_logits_worker, args=(r, world, port, str(p), q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out, t0 = {}, time.time()
    while len(out) < world:
        try:
            r = q.get(timeout=2)
            out[r[0]] = r[1]
        except queue.Empty:
            assert all(pr.is_alive() or pr.exitcode == 0 for pr in procs), "a TP rank crashed"
            assert time.time() - t0 < 300
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0
    for r in range(world):
        got = torch.tensor(out[r])
        assert got.shape == ref.shape
        for i in range(ref.shape[0]):
            rel = float((got[i] - ref[i]).norm() / ref[i].norm())
            cos = float(torch.nn.functional.cosine_similarity(got[i], ref[i], dim=0))
            assert rel <= 1e-2 and cos >= 0.9999, (r, i, rel, cos)


def _argmax_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from localai_amd.models.decoder import TPInfo
        g = torch.Generator().manual_seed(7)
        full = torch.randn(6, 40 * world, generator=g)
        full[1, :] = -float("inf")
        full[1, 40 * world - 1] = 0.0           # the max in the last shard
        full[2, :] = 1.0                        # all tied: the lowest id (rank 0, column 0)
        full[3, 45] = full[3, 5] = 100.0        # tie across the first two shards: id 5
        full[4, 40 * (world - 1)] = 50.0        # first column of the last shard
        tp = TPInfo(rank=rank, world=world, group=dist.group.WORLD)
        got = tp.argmax_cols(full[:, rank * 40:(rank + 1) * 40].contiguous())
        q.put((rank, got.tolist(), full.argmax(-1).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tp_distributed_argmax(world):
    """TPInfo.argmax_cols (the sampler of the TP greedy decode graph) equals the argmax of the
    gathered rows, ties included (lowest id), without gathering them."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_argmax_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, got, ref in res:
        assert got == ref, (got, ref)
    assert res[0][2][2] == 0 and res[0][2][3] == 5
