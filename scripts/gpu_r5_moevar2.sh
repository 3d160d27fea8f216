#!/bin/bash
# MoE decode GEMV variant 1 (two 8-row slots per wave) vs 5 at Mixtral C=1 and C=2
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
run() { LOCALAI_AMD_MOE_GEMV_VAR=$1 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency $3 --max-tokens 128 > gpurun_out/r5_mv2_$2.log 2>&1; }
run 1 c1_v1 1 && run 5 c1_v5 1 && run 1 c1_v1b 1 && run 1 c2_v1 2 && run 5 c2_v5 2 && run 1 c2_v1b 2
rc=$?
kill $HB
exit $rc
