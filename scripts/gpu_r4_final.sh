#!/bin/bash
# round-end rehearsal: the whole GPU suite, smoke, and the driver's default bench
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
# test failures (pytest exit 1) still run smoke and the bench; anything else (timeout, abort) stops here
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/f_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/f_gpu.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step f_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step f_bench.log 600 python -u bench.py
