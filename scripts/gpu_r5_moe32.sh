#!/bin/bash
# moe32 grouped GEMM: numerics tests, then the Mixtral-shaped layer microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_moe32_gpu.py > gpurun_out/r5_moe32_test.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/moe_bench.py --T 64 128 256 > gpurun_out/r5_moe32_bench.log 2>&1
