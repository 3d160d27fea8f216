#!/bin/bash
# Mixtral: HTTP C=256 headline-shaped wave, C=1 MoE GEMV A/B; C=1 Llama profile with the fused norm
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$log | head -20; tail -40 gpurun_out/$log; exit $rc; }; }
step i_mixed.log 600 python -u scripts/mixed_batch_bench.py
grep -h "decode\|sequence" gpurun_out/i_mixed.log | cut -c1-3000
step i_mx1.log 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128
LOCALAI_AMD_MOE_GEMV=0 step i_mx1_old.log 400 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128
step i_mx256.log 700 python -u bench.py --mode http --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/i_prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c1 "Engine C=1, Llama-3-8B Q4_K_M (round 4, fused norm)" --steady 32 --by-grid 32 > $R/gpurun_out/i_prof_c1.md && tail -45 $R/gpurun_out/i_prof_c1.md
