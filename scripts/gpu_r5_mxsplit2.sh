#!/bin/bash
# MoE GEMV splits scaled by the routed pairs (new default): MoE GPU tests + Mixtral C=1 / C=2
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "moe or mixtral or qwen2moe" > gpurun_out/r5_mxs2_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mxs2_c1.log 2>&1 &&
LOCALAI_AMD_MOE_GEMV_SPLITS=2,8 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mxs2_c1_old.log 2>&1 &&
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 2 --max-tokens 128 > gpurun_out/r5_mxs2_c2.log 2>&1 &&
LOCALAI_AMD_MOE_GEMV_SPLITS=2,8 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 2 --max-tokens 128 > gpurun_out/r5_mxs2_c2_old.log 2>&1
rc=$?
kill $HB
exit $rc
