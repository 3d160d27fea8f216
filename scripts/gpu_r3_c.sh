#!/bin/bash
# engine GPU tests after the in-graph penalty ring + C=256 engine bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -m gpu \
  > gpurun_out/r3c_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r3c_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; grep -E "Error|assert" gpurun_out/r3c_tests.log | head -20; exit $rc; fi
timeout -k 10 420 python -u bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r3c_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3c_bench.log
