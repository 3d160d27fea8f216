"""Per-step host control cost of the tensor-parallel engine's replicated scheduling, world 4 on
the CPU: the round-5 path (one gloo TCP broadcast of [n_items, ar_err] per step) against the
/dev/shm channel (parallel/shm_channel.py), both with the follower acknowledging every step.

  python scripts/ctrl_bench.py [--world 4] [--steps 5000]"""
import argparse
import os
import socket
import struct
import time

import torch
import sys

import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, steps, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from localai_amd.parallel.shm_channel import ShmChannel
    ch = ShmChannel.create(dist.group.WORLD, rank, world)
    res = {}
    for name in ("gloo", "shm"):
        dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            if name == "gloo":
                n = torch.tensor([0, 0], dtype=torch.int64)
                dist.broadcast(n, group_src=0)
                int(n[1].item())
            elif rank == 0:
                ch.publish(raw=struct.pack("<qq", 0, 0))
            else:
                struct.unpack_from("<qq", ch.receive(raw=True))
        dist.barrier()
        res[name] = (time.perf_counter() - t0) / steps * 1e6
    if rank == 0:
        q.put(res)
    ch.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5000)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, a.world, port, a.steps, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = q.get(timeout=600)
    for p in ps:
        p.join()
    print(f"world={a.world} steps={a.steps}: per-step control message gloo {res['gloo']:.1f} us, "
          f"shm {res['shm']:.1f} us")


if __name__ == "__main__":
    main()
