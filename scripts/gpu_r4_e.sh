#!/bin/bash
# full GPU suite (regressions), smoke, mixed-batch diagnostics
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
step t_gpu_all.log 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
grep -h "reasons\|decode" gpurun_out/mixed_b.log
