#!/bin/bash
# Mixtral-8x7B C=256 engine decode under rocprofv3 (kernel stats), moe32 grouped GEMM
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_mxprof -o mx -- python3 -u bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 1 --concurrency 256 --max-tokens 128 > gpurun_out/r5_mxprof.log 2>&1
