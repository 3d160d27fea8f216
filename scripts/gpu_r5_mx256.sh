#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe32_gpu.py > gpurun_out/r5_mx256_tests.log 2>&1 || { kill $HB; exit 1; }
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256 --max-tokens 128 > gpurun_out/r5_mx256_new.log 2>&1 || { kill $HB; exit 1; }
LOCALAI_AMD_MOE32_VAR_DOWN=4 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256 --max-tokens 128 > gpurun_out/r5_mx256_v4.log 2>&1
rc=$?
kill $HB
exit $rc
