#!/bin/bash
# MoE decode GEMV variants (LOCALAI_AMD_MOE_GEMV_VAR): correctness test per variant, then Mixtral C=1
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
for v in 21 1 9; do
  LOCALAI_AMD_MOE_GEMV_VAR=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k "moe_gemv" > gpurun_out/r5_mv_test_$v.log 2>&1 || { kill $HB; exit 1; }
done
run() { LOCALAI_AMD_MOE_GEMV_VAR=$1 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mv_$2.log 2>&1; }
run 5 v5 && run 21 v21 && run 1 v1 && run 9 v9 && run 5 v5b && run 21 v21b
rc=$?
kill $HB
exit $rc
