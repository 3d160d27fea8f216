#!/bin/bash
# fused residual-add + RMSNorm in the q|k|v GEMV prologue: numerics, engine C=1 A/B and profile;
# fused TP all-reduce + add + norm (ranks sharing the GPU)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step g_eng.log 600 $PT tests/test_engine_gpu.py -k "fused_norm"
step g_ar.log 500 $PT tests/test_custom_allreduce.py tests/test_tp_gpu.py
step g_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
step g_c1.log 400 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 1 --max-tokens 256
LOCALAI_AMD_GEMV_NORM=0 step g_c1_old.log 400 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 1 --max-tokens 256
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/g_prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c1 "Engine C=1, Llama-3-8B Q4_K_M (round 4, fused norm)" --steady 32 --by-grid 32 > $R/gpurun_out/g_prof_c1.md && tail -45 $R/gpurun_out/g_prof_c1.md
