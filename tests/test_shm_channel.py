"""The tensor-parallel control channel over /dev/shm (parallel/shm_channel.py): sequenced messages
from the leader reach every follower in order and exactly once, including messages larger than the
segment (spilled over the gloo group), at world 3 on the CPU."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from localai_amd.parallel.shm_channel import ShmChannel
    ch = ShmChannel.create(dist.group.WORLD, rank, world, size=64 << 10)
    assert ch is not None
    msgs = [{"i": i, "blob": b"x" * (i * 997 % 5000)} for i in range(300)] + [{"big": b"y" * (200 << 10)}]
    got = []
    for m in msgs:
        if rank == 0:
            ch.publish(m)
        else:
            got.append(ch.receive())
    if rank:
        q.put((rank, got == msgs))
    dist.barrier()
    ch.close()
    dist.destroy_process_group()


def test_shm_channel_in_order_with_spill():
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world - 1))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {1: True, 2: True}
