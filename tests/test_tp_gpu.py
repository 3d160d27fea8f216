"""TP=2 engine on the MI355X with both ranks on the one GPU of the test box (scripts/tp_rehearsal.py):
column/row-parallel layers on the HIP kernels, decode all-reduces through the IPC one-shot kernel,
greedy output agreeing with TP=1.  The ranks are child processes of torch.distributed.run."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world,graphs,overlap,sampling", [(2, True, False, False), (2, True, True, False),
                                                           (4, True, False, False), (2, False, False, False),
                                                           (2, True, False, True), (4, True, False, True)])
def test_tp_engine_ranks_share_one_gpu(tmp_path, world, graphs, overlap, sampling):
    """graphs: decode in captured hipGraphs -- greedy batches on the distributed-argmax graph
    (custom all-reduce kernels only, no RCCL / gloo call inside) -- with every logits row
    compared against TP=1 (scripts/tp_rehearsal.py: cosine >= 0.9999, rel-L2 <= 1e-2).
    overlap: every prefill's row-parallel outputs all-reduced in chunks on the TP comm stream
    (the prefill overlap path, forced on at 2 rows).
    sampling: LocalAI's default sampler (temperature 0.9, top-k 40, top-p 0.95), mirostat 2 and
    repeat-penalised rows, seeded, on the distributed-sampler graph (TPInfo.sample_cols): the rows
    are compared against TP=1 as above, and the drawn tokens share the compared prefix."""
    from localai_amd.models import synth
    p = synth.write_model(str(tmp_path / "tp.gguf"), "tiny-llama", exact=True)
    env = dict(os.environ, TP_REHEARSAL_GRAPHS="1" if graphs else "0", TP_REHEARSAL_SAMPLING="1" if sampling else "0")
    if overlap:
        env.update(LOCALAI_AMD_TP_OVERLAP_ROWS="2", LOCALAI_AMD_TP_OVERLAP_CHUNKS="3")
    port = str(29541 + 8 * world + 4 * int(sampling) + 2 * int(graphs) + int(overlap))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", port,
                        os.path.join(ROOT, "scripts", "tp_rehearsal.py"), p],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "TP_OK" in r.stdout, r.stdout[-2000:]
    print([ln for ln in r.stdout.splitlines() if ln.startswith("TP_ROWS")])
