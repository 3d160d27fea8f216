#!/bin/bash
# A/B: default bench with the full-chunk prefill GEMM tuning vs. without (LOCALAI_AMD_PREFILL_TUNE=0);
# separate TunableOp caches so neither run reuses the other's solutions
mkdir -p gpurun_out
LOCALAI_AMD_CACHE=/tmp/tc_a LOCALAI_AMD_PREFILL_TUNE=0 timeout -k 10 900 python -u bench.py > gpurun_out/b_notune.log 2>&1 || exit 1
tail -1 gpurun_out/b_notune.log
LOCALAI_AMD_CACHE=/tmp/tc_b timeout -k 10 900 python -u bench.py > gpurun_out/b_tune.log 2>&1 || exit 1
tail -1 gpurun_out/b_tune.log
