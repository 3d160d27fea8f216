#!/bin/bash
# multi-step grammar runs: engine GPU tests, then function calling C=32 and the mixed batch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s3h_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed|assert" gpurun_out/s3h_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3h_fc32.log 2>&1; rc=$?; tail -1 gpurun_out/s3h_fc32.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/mixed_batch_bench.py > gpurun_out/s3h_mixed.log 2>&1; rc=$?; grep "decode" gpurun_out/s3h_mixed.log
exit $rc
