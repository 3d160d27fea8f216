#!/bin/bash
# SD pipeline: GPU tests, SD-1.5 512x512 bench with and without the UNet hipGraph
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_sd.py -x -v --timeout 240 --timeout-method thread -m gpu > gpurun_out/sd_test.log 2>&1 && echo SD_TEST_OK &&
timeout -k 10 400 python -u scripts/sd_bench.py --steps 20 --runs 3 > gpurun_out/sd_bench.log 2>&1 && tail -1 gpurun_out/sd_bench.log &&
LOCALAI_AMD_SD_GRAPH=0 timeout -k 10 300 python -u scripts/sd_bench.py --steps 20 --runs 3 > gpurun_out/sd_bench_eager.log 2>&1 && tail -1 gpurun_out/sd_bench_eager.log
