#!/bin/bash
# run-ahead diagnostics: grammar-run counters in FC C=32 and the mixed batch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3k_fc_ra.log 2>&1 || exit $?; grep -E "grammar runs" gpurun_out/s3k_fc_ra.log; tail -1 gpurun_out/s3k_fc_ra.log | cut -c1-140
timeout -k 10 400 python -u scripts/mixed_batch_bench.py > gpurun_out/s3k_mixed_ra.log 2>&1; rc=$?; grep -E "decode|grammar runs" gpurun_out/s3k_mixed_ra.log
exit $rc
