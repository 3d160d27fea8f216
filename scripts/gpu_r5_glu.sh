#!/bin/bash
# 128-row q32 GLU tiles as autotune candidates at M > 128: numerics, then the headline bench with the choices dumped
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_tile_gpu.py -k "q32_glu" > gpurun_out/r5_glu_tests.log 2>&1 || exit $?
BENCH_DUMP_GEMM=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_glu_bench.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_glu_bench2.log 2>&1
