"""Host shared-memory control channel for the ranks of one tensor-parallel group on one node.

The TP engine replicates scheduling: every step, the leader tells the followers what new work
arrived (usually nothing) and the custom all-reduce's error verdict.  Over the gloo control group
that is one TCP broadcast per step on every token's latency path (plus a pickled
broadcast_object_list when work arrives).  Ranks of one node share /dev/shm instead: the leader
writes a sequenced message into a shared segment and each follower spins on the sequence word,
then acknowledges.  SURVEY §2.11 (host-side control plane of intra-node TP); the reference's
llama.cpp RPC backend has no equivalent -- its layer split needs no per-step control message.

Protocol (one writer, world - 1 readers; x86-64 stores become visible in program order):
  header  u64 seq | u64 length | u64 ack[world]        payload  [capacity] bytes
  leader  waits until every ack >= seq - 1 (the previous message has been read), copies the payload,
          writes length, then seq
  reader  spins until seq == expected, copies length bytes, writes ack[rank] = seq
A message larger than the payload region goes over the fallback process group instead (flagged in
the header), so the channel never truncates.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import time
import uuid
from multiprocessing import shared_memory
from typing import Any, Optional

_HDR = 16          # seq, length
_SPILL = 1 << 63   # length flag: the payload went over the process group


class ShmChannel:
    def __init__(self, shm: shared_memory.SharedMemory, rank: int, world: int, owner: bool, group=None,
                 capacity: int = 0):
        self.shm, self.rank, self.world, self.owner, self.group = shm, rank, world, owner, group
        self.buf = shm.buf
        self.ack_off = _HDR
        self.data_off = _HDR + 8 * world
        self.capacity = capacity or (shm.size - self.data_off)
        self.seq = 0
        self.spin_s = float(os.environ.get("LOCALAI_AMD_SHM_SPIN_S", "0.002"))   # busy-wait before yielding

    # ------------------------------------------------------------------ setup
    @classmethod
    def create(cls, group, rank: int, world: int, size: int = 4 << 20) -> Optional["ShmChannel"]:
        """Collective over `group` (gloo): None unless every rank runs on this host (then the
        caller keeps the process-group path)."""
        import torch.distributed as dist
        if os.environ.get("LOCALAI_AMD_SHM_CTRL", "1") == "0" or world < 2:
            return None
        hosts = [None] * world
        dist.all_gather_object(hosts, (socket.gethostname(), os.getpid()), group=group)
        same_host = len({h for h, _ in hosts}) == 1
        name = [f"la_ctrl_{uuid.uuid4().hex[:16]}" if (rank == 0 and same_host) else None]
        dist.broadcast_object_list(name, group_src=0, group=group)
        if not same_host or name[0] is None:
            return None
        ok = 1
        shm = None
        try:
            if rank == 0:
                shm = shared_memory.SharedMemory(name=name[0], create=True, size=size)
                shm.buf[:_HDR + 8 * world] = bytes(_HDR + 8 * world)
            dist.barrier(group=group)
            if rank != 0:
                shm = shared_memory.SharedMemory(name=name[0], create=False)
                try:   # the leader owns the segment: a follower's exit must not unlink it
                    from multiprocessing import resource_tracker
                    resource_tracker.unregister(shm._name, "shared_memory")  # noqa: SLF001
                except Exception:  # noqa: BLE001
                    pass
        except OSError:
            ok = 0
        import torch
        flag = torch.tensor([ok], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if not int(flag.item()):
            if shm is not None:
                shm.close()
                if rank == 0:
                    shm.unlink()
            return None
        return cls(shm, rank, world, rank == 0, group)

    # ------------------------------------------------------------------ data path
    def _u64(self, off: int) -> int:
        return struct.unpack_from("<Q", self.buf, off)[0]

    def _put_u64(self, off: int, v: int) -> None:
        struct.pack_into("<Q", self.buf, off, v)

    def _wait(self, cond) -> None:
        t0 = time.perf_counter()
        while not cond():
            if time.perf_counter() - t0 > self.spin_s:
                time.sleep(0)   # yield once the busy-wait budget is spent (a quiet leader)

    def publish(self, obj: Any = None, raw: Optional[bytes] = None) -> None:
        """Leader: send one message (raw bytes, or a pickled object)."""
        data = raw if raw is not None else pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        seq = self.seq + 1
        acks = [self.ack_off + 8 * r for r in range(1, self.world)]
        self._wait(lambda: all(self._u64(a) >= seq - 1 for a in acks))
        spill = len(data) > self.capacity
        if not spill:
            self.buf[self.data_off:self.data_off + len(data)] = data
        self._put_u64(8, (_SPILL | len(data)) if spill else len(data))
        self._put_u64(0, seq)
        self.seq = seq
        if spill:
            import torch.distributed as dist
            box = [data]
            dist.broadcast_object_list(box, group_src=0, group=self.group)

    def receive(self, raw: bool = False) -> Any:
        """Follower: the next message (blocks until the leader has published it)."""
        seq = self.seq + 1
        self._wait(lambda: self._u64(0) >= seq)
        n = self._u64(8)
        if n & _SPILL:
            import torch.distributed as dist
            box = [None]
            dist.broadcast_object_list(box, group_src=0, group=self.group)
            data = box[0]
        else:
            data = bytes(self.buf[self.data_off:self.data_off + n])
        self._put_u64(self.ack_off + 8 * self.rank, seq)
        self.seq = seq
        return data if raw else pickle.loads(data)

    def close(self) -> None:
        try:
            self.buf = None
            self.shm.close()
            if self.owner:
                self.shm.unlink()
        except Exception:  # noqa: BLE001
            pass
