#!/bin/bash
# Function calling vs plain, C=32, interleaved waves (scripts/fc_bench.py)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u scripts/fc_bench.py --concurrency 32 > gpurun_out/r5_fc32.log 2>&1
