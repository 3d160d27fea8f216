#!/bin/bash
# HTTP headline after burst admission + threaded SSE emit (traced), mixed grammar reasons
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
LOCALAI_AMD_TRACE=gpurun_out/trace_http2.json step b_http_tr2.log 400 python -u bench.py --steps 2 --warmup 1
step b_http_a.log 400 python -u bench.py --steps 5 --warmup 2
LOCALAI_AMD_GIL_SWITCH_MS=0 step b_http_nosw.log 400 python -u bench.py --steps 5 --warmup 2
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
grep -h "reasons\|decode" gpurun_out/mixed_b.log
