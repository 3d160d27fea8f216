#!/bin/bash
# round-end rehearsal on HEAD: whole GPU suite, smoke(), the driver's bench command
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/s3f2_suite.log 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" gpurun_out/s3f2_suite.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3f2_smoke.log 2>&1 || exit $?; tail -1 gpurun_out/s3f2_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s3f2_bench.log 2>&1; rc=$?; tail -1 gpurun_out/s3f2_bench.log | cut -c1-400
exit $rc
