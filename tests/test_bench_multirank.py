"""bench.py's multi-GPU launch contract, rehearsed on the CPU over gloo: `--gpus N` starts its
own N ranks (a torch.distributed.run child), data-parallel replicas report one aggregate JSON
line with n_gpus = N, and `--tp` groups ranks into tensor-parallel replicas."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, *extra):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--preset", "tiny-llama", "--steps", "1", "--warmup", "1",
           "--concurrency", "4", "--prompt-len", "16", "--max-tokens", "8", "--context", "256",
           "--cache-dir", str(tmp_path), "--clients", "1", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("mode", ["engine", "http"])
def test_bench_gpus2_data_parallel(tmp_path, mode):
    out = _bench(tmp_path, "--gpus", "2", "--mode", mode)
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 8
    assert out["steps"] == 1 and out["warmup"] == 1
    # 2 replicas x 4 requests x 8 tokens in the timed wave
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["value"] * out["ms_per_step"] / 1000 == pytest.approx(64, rel=1e-3)


def test_bench_tensor_parallel(tmp_path):
    out = _bench(tmp_path, "--gpus", "2", "--tp", "2", "--mode", "engine")
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp1xtp2"
    assert out["value"] * out["ms_per_step"] / 1000 == pytest.approx(32, rel=1e-3)


def test_bench_dp_times_tp_http(tmp_path):
    out = _bench(tmp_path, "--gpus", "4", "--tp", "2", "--mode", "http")
    assert out["n_gpus"] == 4
    assert out["config"]["parallelism"] == "dp2xtp2"
    assert out["value"] * out["ms_per_step"] / 1000 == pytest.approx(64, rel=1e-3)


def test_bench_gateway_data_parallel(tmp_path):
    """--dp-mode gateway: ONE gateway (rank 0) fronts both engines (rank 1's over backend.proto
    gRPC); it drives concurrency x N streams and reports how many each replica served."""
    out = _bench(tmp_path, "--gpus", "2", "--mode", "http", "--dp-mode", "gateway")
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2-gateway"
    assert out["config"]["global_batch"] == 8
    assert out["value"] * out["ms_per_step"] / 1000 == pytest.approx(64, rel=1e-3)
    served = out["config"]["replica_requests"]
    # warmup + timed wave of 8 requests each, spread over both replicas
    assert sum(served) == 16 and min(served) > 0


def test_bench_http_stream_check_per_request(tmp_path):
    """One HTTP replica: the stream check adds up events + merged (held-back) tokens to the
    reported count per request and passes on a well-formed stream."""
    out = _bench(tmp_path, "--mode", "http")
    sc = out["stream_check"]
    assert sc["reported_tokens"] == sc["expected_tokens"] == 4 * 8
    assert (sc["streamed_events"] - sc["split_events"] + sc["merged_tokens"] + sc["tail_tokens"]
            == sc["reported_tokens"]), sc
    assert sc["bad_streams"] == 0 and sc["short_requests"] == 0


def test_bench_open_loop_arrivals(tmp_path):
    """--arrival-rate: open-loop Poisson arrivals over HTTP report tokens/s, TTFT and inter-token
    latency percentiles, with the same wire accounting."""
    out = _bench(tmp_path, "--mode", "http", "--arrival-rate", "50", "--requests", "6")
    assert out["requests"] == 6 and out["tokens_per_s"] > 0
    assert out["p99_ttft_ms"] >= out["p50_ttft_ms"] > 0
    assert out["p99_itl_ms"] >= out["p50_itl_ms"] > 0
    sc = out["stream_check"]
    assert sc["reported_tokens"] == sc["expected_tokens"] == 6 * 8
    assert (sc["streamed_events"] - sc["split_events"] + sc["merged_tokens"] + sc["tail_tokens"]
            == sc["reported_tokens"]) and sc["bad_streams"] == 0
