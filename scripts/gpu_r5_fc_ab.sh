#!/bin/bash
# Function calling vs plain (C=32, 8 interleaved waves): grammar run-ahead policies
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 500 python -u scripts/fc_bench.py --concurrency 32 --waves 6 > gpurun_out/r5_fc_base.log 2>&1 || exit $?
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 timeout -k 10 500 python -u scripts/fc_bench.py --concurrency 32 --waves 6 > gpurun_out/r5_fc_ra.log 2>&1 || exit $?
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 LOCALAI_AMD_GRAMMAR_MIXED_FRAC=1.0 LOCALAI_AMD_GRAMMAR_MIXED_K=8 timeout -k 10 500 python -u scripts/fc_bench.py --concurrency 32 --waves 6 > gpurun_out/r5_fc_ra8.log 2>&1
