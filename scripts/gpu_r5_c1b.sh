#!/bin/bash
# batch-1 decode: fused residual+norm q|k|v prologue with fewer down-projection split-K slabs
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --mode engine --steps 3 --warmup 1 --max-tokens 256 --concurrency 1"
timeout -k 10 400 $B > gpurun_out/r5_c1b_base.log 2>&1 || exit $?
LOCALAI_AMD_GEMV_NORM=1 LOCALAI_AMD_GEMV_MAX_SPLITS=2 timeout -k 10 400 $B > gpurun_out/r5_c1b_n2.log 2>&1 || exit $?
LOCALAI_AMD_GEMV_NORM=1 LOCALAI_AMD_GEMV_MAX_SPLITS=4 timeout -k 10 400 $B > gpurun_out/r5_c1b_n4.log 2>&1 || exit $?
LOCALAI_AMD_GEMV_MAX_SPLITS=4 timeout -k 10 400 $B > gpurun_out/r5_c1b_s4.log 2>&1 || exit $?
timeout -k 10 400 $B > gpurun_out/r5_c1b_base2.log 2>&1
