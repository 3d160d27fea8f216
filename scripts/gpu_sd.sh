#!/bin/bash
# SD pipeline: GPU tests (fused GroupNorm kernel + pipeline), SD-1.5 512x512 bench NHWC / NCHW,
# rocprof kernel stats of one 10-step image
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_sd.py -x -v --timeout 240 --timeout-method thread -m gpu > gpurun_out/sd_test.log 2>&1 && echo SD_TEST_OK &&
timeout -k 10 400 python -u scripts/sd_bench.py --steps 20 --runs 3 > gpurun_out/sd_bench.log 2>&1 && tail -1 gpurun_out/sd_bench.log &&
timeout -k 10 300 python -u scripts/sd_bench.py --steps 20 --runs 3 --nchw > gpurun_out/sd_bench_nchw.log 2>&1 && tail -1 gpurun_out/sd_bench_nchw.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sd -o sd -- python3 scripts/sd_bench.py --steps 10 --runs 1 > gpurun_out/prof_sd.log 2>&1 && echo PROF_OK
