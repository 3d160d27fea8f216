#!/bin/bash
# burst prefill-first (default) vs mixed prefill + decode steps, same box, alternated
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_pf_on.log 2>&1 || exit $?
LOCALAI_AMD_PREFILL_FIRST_MS=0 timeout -k 10 500 python -u bench.py > gpurun_out/r5_pf_off.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_pf_on2.log 2>&1 || exit $?
LOCALAI_AMD_PREFILL_FIRST_MS=0 timeout -k 10 500 python -u bench.py > gpurun_out/r5_pf_off2.log 2>&1
