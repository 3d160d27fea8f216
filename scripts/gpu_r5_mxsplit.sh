#!/bin/bash
# Mixtral C=1: split-K of the MoE decode GEMVs (gate|up, down); default = dense heuristic (2, 8)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
run() { LOCALAI_AMD_MOE_GEMV_SPLITS=$1 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mxs_$2.log 2>&1; }
run 2,2 d2 && run 2,4 d4b && run 2,7 d7 && run 0,0 def3 && run 2,4 d4c && run 2,2 d2b
rc=$?
kill $HB
exit $rc
