#!/bin/bash
# grammar: state-key fix + one-level transition expansion; default vs run-ahead, FC C=32 and mixed batch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k grammar -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s3j_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/s3j_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3j_fc.log 2>&1 || exit $?; tail -1 gpurun_out/s3j_fc.log | cut -c1-140
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 timeout -k 10 300 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3j_fc_ra.log 2>&1 || exit $?; tail -1 gpurun_out/s3j_fc_ra.log | cut -c1-140
timeout -k 10 400 python -u scripts/mixed_batch_bench.py > gpurun_out/s3j_mixed.log 2>&1 || exit $?; grep "decode" gpurun_out/s3j_mixed.log
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 timeout -k 10 400 python -u scripts/mixed_batch_bench.py > gpurun_out/s3j_mixed_ra.log 2>&1; rc=$?; grep "decode" gpurun_out/s3j_mixed_ra.log
exit $rc
