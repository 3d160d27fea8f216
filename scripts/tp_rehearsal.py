"""Tensor-parallel engine rehearsal on ONE GPU: WORLD ranks (torch.distributed.run) share cuda:0,
the control plane and the prefill all-gathers run over gloo, the decode all-reduces over the
one-shot IPC kernel (parallel/custom_ar.py) -- the TP code path of an 8-GPU node on real HIP
kernels.

Decode runs in captured hipGraphs (use_graphs=True): greedy batches take the distributed-argmax
graph (LLMEngine._capture(tp_greedy=True)), whose only collectives are the custom all-reduce
kernels (layer boundaries + the B x world candidate exchange), so the graph holds no RCCL / gloo
call.  Rank 0 compares EVERY logits row of the TP run (prefill row + each decode step, gathered
off the graph) with a TP=1 engine's rows for the same prefix: cosine >= 0.9999 and rel-L2 <= 1e-2
on every row up to the first token where the two greedy streams part (a near-tie resolved
differently by the reordered sums), and at least MIN_ROWS rows compared per prompt.  Prints TP_OK."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MIN_ROWS = 4


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    from localai_amd.models.decoder import TPInfo
    from localai_amd.parallel.custom_ar import maybe_create
    path = sys.argv[1]
    graphs = os.environ.get("TP_REHEARSAL_GRAPHS", "1") == "1"
    tp = TPInfo(rank=rank, world=world, group=dist.group.WORLD)
    tp.car = maybe_create(dist.group.WORLD, rank, world, "cuda:0")
    ctrl = dist.new_group(backend="gloo")
    cfg = dict(model_path=path, device="cuda:0", context_size=256, max_num_seqs=4, use_graphs=graphs,
               record_tokens=True, record_logits=True)
    eng = LLMEngine(EngineConfig(**cfg), tp=tp, ctrl_group=ctrl)
    prompts = ["tensor parallel on one gpu", "second prompt"]
    n_tok = 12
    sampling = os.environ.get("TP_REHEARSAL_SAMPLING", "0") == "1"
    if sampling:
        # LocalAI's default sampler (temperature 0.9, top-k 40, top-p 0.95) on the first prompt,
        # mirostat 2 on the second, seeded: the TP run must draw the TP=1 tokens
        prompts = ["tensor parallel on one gpu", "mirostat prompt", "penalised prompt"]
        kws = [dict(temperature=0.9, top_k=40, top_p=0.95, seed=1234),
               dict(temperature=0.9, mirostat=2, mirostat_tau=5.0, mirostat_eta=0.1, seed=99),
               dict(temperature=0.8, top_k=20, repeat_penalty=1.3, seed=7)]
        sps = iter([SamplingParams(max_tokens=n_tok, ignore_eos=True, **k) for k in kws * 2])
        sp = lambda: next(sps)  # noqa: E731
    else:
        sp = lambda: SamplingParams(max_tokens=n_tok, temperature=0.0, ignore_eos=True)  # noqa: E731
    if rank == 0:
        outs = [eng.generate(p, sp()) for p in prompts]
        tpg_graphs = len(eng._graphs_tpg)
        tps_graphs = len(eng._graphs_tps)
        eng.shutdown()
        single = LLMEngine(EngineConfig(**cfg))
        refs = [single.generate(p, sp()) for p in prompts]
        print("TP texts", [o["text"] for o in outs], "single", [r["text"] for r in refs], flush=True)
        assert all(o["completion_tokens"] == n_tok for o in outs)
        if graphs and not sampling:
            assert tpg_graphs > 0, "greedy TP decode did not run the distributed-argmax graph"
        if graphs and sampling:
            assert tps_graphs > 0, "sampled TP decode did not run the distributed-sampler graph"
        worst_cos, worst_rel, total = 1.0, 0.0, 0
        for o, r in zip(outs, refs):
            a_ids, b_ids = o["token_ids"], r["token_ids"]
            la, lb = o["logits"], r["logits"]
            assert len(la) == len(a_ids) and len(lb) == len(b_ids), (len(la), len(a_ids), len(lb), len(b_ids))
            rows = 0
            for j in range(min(len(a_ids), len(b_ids))):
                x, y = la[j].float().cpu(), lb[j].float().cpu()
                assert x.shape == y.shape, (x.shape, y.shape)
                cos = float(torch.nn.functional.cosine_similarity(x, y, dim=0))
                rel = float((x - y).norm() / y.norm())
                worst_cos, worst_rel = min(worst_cos, cos), max(worst_rel, rel)
                assert cos >= 0.9999 and rel <= 1e-2, (j, cos, rel)
                rows += 1
                if a_ids[j] != b_ids[j]:
                    break  # the prefixes differ from here on
            # a sampled stream may part at any draw whose uniform falls within the logits' rounding
            # difference of a CDF boundary; the sampler itself is pinned on identical logits in
            # tests/test_tp_sample_gpu.py, so here only the rows up to the parting are compared
            assert rows >= (1 if sampling else MIN_ROWS), f"only {rows} rows share a prefix with TP=1"
            total += rows
        assert tp.car is not None and not tp.car.timed_out(), "custom all-reduce unavailable or timed out"
        same = sum(int(o["token_ids"] == r["token_ids"]) for o, r in zip(outs, refs))
        if sampling:
            assert same >= 1 and total >= MIN_ROWS * len(outs) // 2, (same, total)
        print(f"TP_ROWS world={world} graphs={graphs} sampling={sampling} rows={total} worst_cos={worst_cos:.6f} "
              f"worst_rel={worst_rel:.2e} identical_streams={same}/{len(outs)}", flush=True)
        print("TP_OK", flush=True)
    else:
        eng.run_follower()
    if tp.car is not None:
        tp.car.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
