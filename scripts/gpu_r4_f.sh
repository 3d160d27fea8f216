#!/bin/bash
# re-run of the round's GPU failures + MoE GEMV numerics + Mixtral C=1 decode A/B
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step t_moe.log 300 $PT tests/test_kernels_gpu.py -k "moe or clip"
step t_fix.log 600 $PT tests/test_engine_gpu.py -k "penalties or rides or stride or mixtral"
step t_xl.log 300 $PT tests/test_sdxl.py -k "fp32_forward or graph_matches"
step t_ar8.log 400 $PT tests/test_custom_allreduce.py
step mx1.log 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128
LOCALAI_AMD_MOE_GEMV=0 step mx1_old.log 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128
step fc8.log 500 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32
LOCALAI_AMD_GRAMMAR_RUN_AHEAD=1 step fc8_ra.log 500 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
grep -h "reasons\|decode" gpurun_out/mixed_b.log
