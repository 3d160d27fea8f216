"""One-shot IPC all-reduce (ops/csrc/allreduce.hip, parallel/custom_ar.py) with two ranks sharing
the one GPU of the test box: exact sums, mixed sizes, graph replay (scripts/ar_check.py).  The
ranks run as child processes of torch.distributed.run, started from here."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_ranks_share_one_gpu(world):
    """2, 4 and 8 ranks (the 8-GPU node's TP=8 epoch protocol and 7-peer read pattern) sharing the
    test box's GPU: one-shot and two-shot sums, graph replay, and a late peer's timeout reaching
    every rank's error word."""
    # one hardware queue per rank: 8 processes x HIP's default 4 queues oversubscribe the GPU's
    # hardware queues, so a peer's kernel could wait for a queue time slice while the others spin
    # (a timeout on a shared device; separate GPUs never have it)
    env = dict(os.environ, LOCALAI_AMD_AR_SAME_GPU="1", GPU_MAX_HW_QUEUES="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(29533 + world),
                        os.path.join(ROOT, "scripts", "ar_check.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        # the failing rank's traceback, not just torchrun's summary
        lines = [ln for ln in r.stderr.splitlines() if "Gloo" not in ln]
        tb = [i for i, ln in enumerate(lines) if "Traceback" in ln]
        head = "\n".join(lines[tb[0]:tb[0] + 40]) if tb else ""
        raise AssertionError(head + "\n---\n" + r.stdout[-2000:] + r.stderr[-1500:])
    assert "AR_OK" in r.stdout, r.stdout[-2000:]


def test_tpinfo_falls_back_without_custom_ar():
    """CPU / gloo TP groups never get a CustomAllReduce (maybe_create returns None)."""
    from localai_amd.parallel.custom_ar import maybe_create
    assert maybe_create(None, 0, 2, "cpu") is None
    assert maybe_create(None, 0, 1, "cuda:0") is None
