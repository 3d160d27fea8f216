"""TP=2 engine on the MI355X with both ranks on the one GPU of the test box (scripts/tp_rehearsal.py):
column/row-parallel layers on the HIP kernels, decode all-reduces through the IPC one-shot kernel,
greedy output agreeing with TP=1.  The ranks are child processes of torch.distributed.run."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world,graphs,overlap", [(2, True, False), (2, True, True), (4, True, False),
                                                  (2, False, False)])
def test_tp_engine_ranks_share_one_gpu(tmp_path, world, graphs, overlap):
    """graphs: decode in captured hipGraphs -- greedy batches on the distributed-argmax graph
    (custom all-reduce kernels only, no RCCL / gloo call inside) -- with every logits row
    compared against TP=1 (scripts/tp_rehearsal.py: cosine >= 0.9999, rel-L2 <= 1e-2).
    overlap: every prefill's row-parallel outputs all-reduced in chunks on the TP comm stream
    (the prefill overlap path, forced on at 2 rows)."""
    from localai_amd.models import synth
    p = synth.write_model(str(tmp_path / "tp.gguf"), "tiny-llama", exact=True)
    env = dict(os.environ, TP_REHEARSAL_GRAPHS="1" if graphs else "0")
    if overlap:
        env.update(LOCALAI_AMD_TP_OVERLAP_ROWS="2", LOCALAI_AMD_TP_OVERLAP_CHUNKS="3")
    port = str(29541 + 4 * world + 2 * int(graphs) + int(overlap))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", port,
                        os.path.join(ROOT, "scripts", "tp_rehearsal.py"), p],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "TP_OK" in r.stdout, r.stdout[-2000:]
    print([ln for ln in r.stdout.splitlines() if ln.startswith("TP_ROWS")])
