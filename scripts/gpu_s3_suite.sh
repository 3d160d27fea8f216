#!/bin/bash
# Parler-TTS GPU test first, then the whole GPU suite (round-end rehearsal)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parler.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s3_parler.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/s3_parler.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/s3_suite.log 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" gpurun_out/s3_suite.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s3_fc32.log 2>&1; rc=$?; tail -1 gpurun_out/s3_fc32.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/mixed_batch_bench.py > gpurun_out/s3_mixed.log 2>&1; rc=$?; grep "decode" gpurun_out/s3_mixed.log
exit $rc
