"""Tensor-parallel engine rehearsal on ONE GPU: two ranks (torch.distributed.run) share cuda:0,
the control plane and the all-gathers run over gloo, the decode all-reduces over the one-shot
IPC kernel (parallel/custom_ar.py) -- the TP=2 code path of an 8-GPU node on real HIP kernels.
Rank 0 generates greedily; the follower mirrors every step; rank 0 compares with a TP=1 engine
and prints TP_OK.  Eager mode (gloo collectives are not graph-capturable)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    tp = TPInfo(rank=rank, world=world, group=dist.group.WORLD)
    tp.car = maybe_create(dist.group.WORLD, rank, world, "cuda:0")
    ctrl = dist.new_group(backend="gloo")
    cfg = dict(model_path=path, device="cuda:0", context_size=256, max_num_seqs=4, use_graphs=False)
    eng = LLMEngine(EngineConfig(**cfg), tp=tp, ctrl_group=ctrl)
    prompts = ["tensor parallel on one gpu", "second prompt"]
    sp = lambda: SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)  # noqa: E731
    if rank == 0:
        outs = [eng.generate(p, sp()) for p in prompts]
        eng.shutdown()
        single = LLMEngine(EngineConfig(**cfg))
        refs = [single.generate(p, sp()) for p in prompts]
        print("TP texts", [o["text"] for o in outs], "single", [r["text"] for r in refs], flush=True)
        assert all(o["completion_tokens"] == 8 for o in outs)
        # sharded bf16 reductions reorder sums: the first token must agree
        assert all(o["text"][:1] == r["text"][:1] for o, r in zip(outs, refs)), "TP and TP=1 diverge at token 1"
        assert tp.car is not None and not tp.car.timed_out(), "custom all-reduce unavailable or timed out"
        print("TP_OK", flush=True)
    else:
        eng.run_follower()
    if tp.car is not None:
        tp.car.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
