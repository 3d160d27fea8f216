#!/bin/bash
# grammar: default path (in-graph masks, single step) vs run-ahead opt-in; FC C=32 twice each
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k grammar -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s3i_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/s3i_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3i_fc32_$i.log 2>&1 || exit $?; tail -1 gpurun_out/s3i_fc32_$i.log | cut -c1-160
done
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 timeout -k 10 300 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3i_fc32_ra.log 2>&1 || exit $?; tail -1 gpurun_out/s3i_fc32_ra.log | cut -c1-160
timeout -k 10 600 python -u scripts/mixed_batch_bench.py > gpurun_out/s3i_mixed.log 2>&1; rc=$?; grep "decode" gpurun_out/s3i_mixed.log
exit $rc
