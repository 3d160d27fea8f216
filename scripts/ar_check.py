"""Two-or-more-rank check of the one-shot IPC all-reduce (parallel/custom_ar.py): exact rank-ordered
sums for fp32 / bf16 messages of 1, 3 and 64 decode rows, a ragged tail and the largest size,
back-to-back calls of different sizes, and replay inside a captured hipGraph.  Launch with
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/ar_check.py
Every rank may share one GPU (LOCALAI_AMD_AR_SAME_GPU=1): the buffers are then IPC-mapped inside
one device, which exercises the whole protocol except the xGMI transport itself."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from localai_amd.parallel.custom_ar import CustomAllReduce


def inputs(rank, n, dtype, dev, call):
    g = torch.Generator(device="cpu").manual_seed(1000 * call + rank)
    return torch.randn(n, generator=g).to(dtype).to(dev)


def expected(world, n, dtype, dev, call):
    acc = torch.zeros(n, dtype=torch.float32, device=dev)
    for r in range(world):
        acc += inputs(r, n, dtype, dev, call).float()
    return acc.to(dtype)


def make_car(rank, world, dev):
    """One setup attempt: the regions are uncached whole-granule allocations (custom_ar._alloc),
    and any rank's failure raises on every rank with the region, pointer and allocation base."""
    return CustomAllReduce(dist.group.WORLD, rank, world, dev)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if os.environ.get("LOCALAI_AMD_AR_SAME_GPU") == "1" else int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    car = make_car(rank, world, dev)
    if os.environ.get("LOCALAI_AMD_AR_SAME_GPU") == "1":
        # every rank on ONE device: 8 processes x 4 HIP queues oversubscribe the hardware queues,
        # so a peer's kernel may wait for a time slice while this one spins -- allow ~16 s
        # instead of ~1 s before a wait counts as a dead peer (separate GPUs never need it)
        car.SPIN_LIMIT = 1 << 24
    cases = [(4096, torch.float32), (3 * 4096, torch.float32), (4096, torch.bfloat16), (1000, torch.float32),
             (64 * 4096, torch.float32), (car.max_elems, torch.bfloat16), (4096 + 8, torch.bfloat16),
             # two-shot (reduce-scatter + all-gather) past the one-shot's size: a decode batch of 256
             # rows of 4096 (fp32 and bf16), a ragged size, the largest size
             (256 * 4096, torch.float32), (256 * 4096, torch.bfloat16), (car.max_elems + 1000 + 3, torch.float32),
             (car.max_elems2, torch.bfloat16)]
    for call, (n, dt) in enumerate(cases):
        t = inputs(rank, n, dt, dev, call)
        car.all_reduce(t)
        torch.cuda.synchronize()
        ref = expected(world, n, dt, dev, call)
        err = (t.float() - ref.float()).abs().max().item()
        assert err == 0.0, (rank, n, dt, err, "timed out" if car.error_flag() else "no timeout")
    # graph capture: calls of mixed sizes (one-shot and two-shot), replayed twice with fresh inputs
    gcases = cases[:3] + [cases[7]]
    bufs = [torch.empty(n, dtype=dt, device=dev) for n, dt in gcases]
    srcs = [torch.empty_like(b) for b in bufs]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for b, src in zip(bufs, srcs):
                b.copy_(src)
                car.all_reduce(b)
    torch.cuda.current_stream().wait_stream(s)
    for rep in range(2):
        for i, (n, dt) in enumerate(gcases):
            srcs[i].copy_(inputs(rank, n, dt, dev, 100 + 10 * rep + i))
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        for i, (n, dt) in enumerate(gcases):
            ref = expected(world, n, dt, dev, 100 + 10 * rep + i)
            assert (bufs[i].float() - ref.float()).abs().max().item() == 0.0, (rank, "graph", rep, i,
                                                                               "timed out" if car.error_flag() else
                                                                               "no timeout")
    assert not car.timed_out()
    # fused all-reduce + bias + residual + norm (CustomAllReduce.add_norm), interleaved with plain
    # one-shot calls on the same channels: residual exact, normed row within bf16 rounding
    def an_case(call, M, D, S, mode, with_bias):
        g0 = torch.Generator().manual_seed(5000 + call)            # shared by all ranks
        res = torch.randn(M, D, generator=g0)
        w = torch.rand(D, generator=g0) + 0.5
        nb = torch.randn(D, generator=g0) * 0.1 if mode == 1 else None
        bias = torch.randn(D, generator=g0) * 0.1 if with_bias else None
        tot = torch.zeros(M, D)
        for r in range(world):
            gr = torch.Generator().manual_seed(6000 + 10 * call + r)
            loc = torch.randn(max(S, 1), M, D, generator=gr)
            acc = loc[0].clone()
            for k in range(1, S):
                acc = acc + loc[k]                                 # the kernel's slab order
            wire = acc.to(torch.bfloat16)
            tot += wire.float()
            if r == rank:
                part = ops.Partial(loc.to(dev) if S else wire.to(dev))
        ref_res = res + (tot + (bias if bias is not None else 0.0))
        if mode == 0:
            ref = ref_res * torch.rsqrt(ref_res.pow(2).mean(-1, keepdim=True) + 1e-5) * w
        else:
            mu = ref_res.mean(-1, keepdim=True)
            ref = (ref_res - mu) * torch.rsqrt((ref_res - mu).pow(2).mean(-1, keepdim=True) + 1e-5) * w + nb
        rd = res.to(dev)
        out = car.add_norm(part, None if bias is None else bias.to(dev), rd, w.to(dev),
                           None if nb is None else nb.to(dev), 1e-5, mode)
        torch.cuda.synchronize()
        assert torch.allclose(rd.cpu(), ref_res, rtol=0, atol=1e-5), (rank, "add_norm residual", call)
        err = (out.float().cpu() - ref).abs().max().item()
        assert err < 2e-2 * max(1.0, ref.abs().max().item()), (rank, "add_norm out", call, err)
    from localai_amd import ops
    an_case(0, 1, 4096, 3, 0, True)
    t = inputs(rank, 3 * 4096, torch.float32, dev, 40)          # one-shot on overlapping channels
    car.all_reduce(t)
    an_case(1, 3, 256, 0, 1, False)
    an_case(2, 2, 8192, 9, 0, False)
    an_case(3, 64, 4096, 1, 0, True)
    torch.cuda.synchronize()
    assert (t.float() - expected(world, 3 * 4096, torch.float32, dev, 40).float()).abs().max().item() == 0.0
    assert not car.timed_out()
    # latency of one decode row (same-GPU numbers say nothing about xGMI; recorded for reference)
    t = inputs(rank, 4096, torch.float32, dev, 7)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        car.all_reduce(t)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 200 * 1e6
    t = inputs(rank, 256 * 4096, torch.float32, dev, 8)   # a 256-row decode batch: two-shot
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        car.all_reduce(t)
    torch.cuda.synchronize()
    us2 = (time.perf_counter() - t0) / 50 * 1e6
    dist.barrier()
    car.close()
    # a late peer: rank 1 arrives ~1.5 s after rank 0, whose spin limit is tiny -> rank 0's wait
    # times out; the per-step agreement (TPInfo.check_custom_ar) must fail loudly on EVERY rank
    # and drop the custom path, never hand out the stale sum silently
    from localai_amd.models.decoder import CustomAllReduceTimeout, TPInfo
    car2 = make_car(rank, world, dev)
    car2.SPIN_LIMIT = 1 << 8
    tpi = TPInfo(rank=rank, world=world, group=dist.group.WORLD, car=car2)
    t = inputs(rank, 4096, torch.float32, dev, 9)
    dist.barrier()
    if rank == 1:
        time.sleep(1.5)
    tpi.all_reduce(t)
    torch.cuda.synchronize()
    dist.barrier()
    # the timed-out wait wrote EVERY rank's error word (allreduce.hip): no collective needed to
    # learn about it, so the engine reads only its own word after the step's token readback
    assert car2.error_flag(), (rank, "error word not set by the peer's timeout")
    raised = False
    try:
        tpi.check_custom_ar(dist.group.WORLD)
    except CustomAllReduceTimeout:
        raised = True
    assert raised and tpi.car is None, (rank, raised)
    t2 = inputs(rank, 4096, torch.float32, dev, 10)
    tpi.all_reduce(t2)          # now RCCL/gloo path: exact again
    ref = expected(world, 4096, torch.float32, torch.device("cpu"), 10)
    assert (t2.float().cpu() - ref).abs().max().item() < 1e-5, rank
    dist.barrier()
    if rank == 0:
        print(f"AR_OK world={world} one-row all-reduce {us:.1f} us/call, 256-row (4 MiB fp32, two-shot) "
              f"{us2:.1f} us/call")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
