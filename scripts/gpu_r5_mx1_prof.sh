#!/bin/bash
# Mixtral-8x7B C=1 engine decode under rocprofv3 (kernel stats)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_mx1prof -o mx1 -- python3 -u bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mx1prof.log 2>&1
rc=$?
kill $HB
exit $rc
