#!/bin/bash
# headline bench: 16 vs 32 device decode steps per host round trip (A/B, alternating)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-300; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
for k in 0 32 0 32; do
  BENCH_DECODE_STEPS=$k step x_k$k.log 500 python -u bench.py --steps 4 --warmup 1
done
