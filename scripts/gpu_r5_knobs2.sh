#!/bin/bash
# Llama: GIL switch 5 ms, with / without admission at 4096 tokens; Mixtral: prefill-first cap 2 s vs 0.4 s
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
LOCALAI_AMD_GIL_SWITCH_MS=5 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k2_gil5.log 2>&1 &&
LOCALAI_AMD_GIL_SWITCH_MS=5 LOCALAI_AMD_ADMIT_TOKENS=4096 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k2_gil5adm.log 2>&1 &&
LOCALAI_AMD_GIL_SWITCH_MS=5 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k2_gil5b.log 2>&1 &&
LOCALAI_AMD_GIL_SWITCH_MS=5 LOCALAI_AMD_ADMIT_TOKENS=4096 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k2_gil5admb.log 2>&1 &&
timeout -k 10 900 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_k2_mx_def.log 2>&1 &&
LOCALAI_AMD_PREFILL_FIRST_MS=2000 timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_k2_mx_pf2.log 2>&1 &&
timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_k2_mx_def2.log 2>&1 &&
LOCALAI_AMD_PREFILL_FIRST_MS=2000 timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_k2_mx_pf22.log 2>&1
rc=$?
kill $HB
exit $rc
