#!/bin/bash
# batch-1 / batch-2 decode: in-kernel split-K reduction in the GEMV (default) vs off, and with the
# fused residual+norm q|k|v prologue
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or dp4" > gpurun_out/r5_c1_tests.log 2>&1 || exit $?
B="python -u bench.py --mode engine --steps 3 --warmup 1 --max-tokens 256"
for C in 1 2; do
  timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_c${C}_red.log 2>&1 || exit $?
  LOCALAI_AMD_GEMV_REDUCE=0 timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_c${C}_nored.log 2>&1 || exit $?
  LOCALAI_AMD_GEMV_NORM=1 timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_c${C}_rednorm.log 2>&1 || exit $?
done
