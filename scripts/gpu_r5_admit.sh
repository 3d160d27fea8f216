#!/bin/bash
# admission window closing once one prefill chunk is waiting (default) vs the round-4 window
set -o pipefail
mkdir -p gpurun_out
BENCH_ARRIVALS=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_adm_on.log 2>&1 || exit $?
BENCH_ARRIVALS=1 LOCALAI_AMD_ADMIT_TOKENS=0 timeout -k 10 500 python -u bench.py > gpurun_out/r5_adm_off.log 2>&1 || exit $?
BENCH_ARRIVALS=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_adm_on2.log 2>&1 || exit $?
BENCH_ARRIVALS=1 LOCALAI_AMD_ADMIT_TOKENS=0 timeout -k 10 500 python -u bench.py > gpurun_out/r5_adm_off2.log 2>&1
