#!/bin/bash
# Llama-3-8B C=1: GEMV split-K cap (all decode GEMVs) 4 / 2 vs the heuristic
set -o pipefail
mkdir -p gpurun_out
run() { LOCALAI_AMD_GEMV_MAX_SPLITS=$1 timeout -k 10 400 python -u bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 256 > gpurun_out/r5_c1cap_$2.log 2>&1; }
run 0 def && run 4 cap4 && run 2 cap2 && run 0 def2 && run 4 cap4b
