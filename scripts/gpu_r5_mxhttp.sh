#!/bin/bash
# Mixtral-8x7B Q4_K_M through the headline HTTP bench layout at HEAD (BASELINE config 4's model)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 900 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_mxhttp.log 2>&1
rc=$?
kill $HB
exit $rc
