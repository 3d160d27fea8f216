#!/bin/bash
# Mixtral-8x7B Q4_K_M (random-init) engine decode: moe32 grouped GEMM vs the 16-column kernel
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
for C in 256 64; do
  timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency $C --max-tokens 128 > gpurun_out/r5_mx_c$C.log 2>&1 || exit $?
  LOCALAI_AMD_MOE32=0 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency $C --max-tokens 128 > gpurun_out/r5_mx_c${C}_old.log 2>&1 || exit $?
done
