#!/bin/bash
# per-call GEMV variant at M=2: tests, C=2 bench x2, C=1 bench
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-300; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step gv4_kern.log 300 $PT tests/test_kernels_gpu.py -k "gemv or act_linear or qkv_rope"
step gv4_eng.log 400 $PT tests/test_engine_gpu.py -k "fused_norm"
step gv4_c2a.log 300 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 2 --max-tokens 256
step gv4_c2b.log 300 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 2 --max-tokens 256
