#!/bin/bash
# constrained rows hand their run tokens to the scheduler as a computed run: grammar tests, mixed wave, FC C=32
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step j_eng.log 600 $PT tests/test_engine_gpu.py -k "grammar or fused_norm or spec or draft"
step j_mixed.log 600 python -u scripts/mixed_batch_bench.py
grep -h "decode\|sequence" gpurun_out/j_mixed.log | cut -c1-3000
step j_fc8.log 500 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32
