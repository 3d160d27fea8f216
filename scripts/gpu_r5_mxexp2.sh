#!/bin/bash
# device memory with / without the resident bf16 expert copies (Mixtral HTTP C=256)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
LOCALAI_AMD_PREFILL_BF16_EXPERTS=0 timeout -k 10 900 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_mxe_off2.log 2>&1 &&
timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_mxe_on3.log 2>&1
rc=$?
kill $HB
exit $rc
