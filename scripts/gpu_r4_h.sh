#!/bin/bash
# fused norm (batch-1/2) + fused TP AR/norm + grammar expansion policy: tests, C=1 A/B, mixed wave, FC C=32
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step h_eng.log 600 $PT tests/test_engine_gpu.py -k "fused_norm or grammar"
step h_ar.log 500 $PT tests/test_custom_allreduce.py tests/test_tp_gpu.py
step h_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step h_c1.log 400 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 1 --max-tokens 256
LOCALAI_AMD_GEMV_NORM=0 step h_c1_old.log 400 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 1 --max-tokens 256
step h_mixed.log 600 python -u scripts/mixed_batch_bench.py
grep -h "decode\|reasons" gpurun_out/h_mixed.log | cut -c1-600
step h_fc8.log 500 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32
