#!/bin/bash
# AR world 2/4/8 with one HW queue per rank, TP engine, smoke, driver-default bench
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step r_ar.log 600 $PT tests/test_custom_allreduce.py tests/test_tp_gpu.py tests/test_sd.py -k "allreduce or tp2 or after_diffusion"
step r_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step r_bench.log 600 python -u bench.py
