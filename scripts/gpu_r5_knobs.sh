#!/bin/bash
# serving knobs at HEAD, alternated: default / admission closes at 4096 queued tokens / GIL switch 5 ms
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_def.log 2>&1 &&
LOCALAI_AMD_ADMIT_TOKENS=4096 timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_adm4k.log 2>&1 &&
LOCALAI_AMD_GIL_SWITCH_MS=5 timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_gil5.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_def2.log 2>&1 &&
LOCALAI_AMD_ADMIT_TOKENS=4096 timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_adm4k2.log 2>&1 &&
LOCALAI_AMD_GIL_SWITCH_MS=5 timeout -k 10 500 python -u bench.py > gpurun_out/r5_kn_gil52.log 2>&1
