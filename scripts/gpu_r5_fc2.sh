#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -k grammar -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_fc2_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/fc_bench.py --concurrency 32 --waves 6 > gpurun_out/r5_fc2.log 2>&1
