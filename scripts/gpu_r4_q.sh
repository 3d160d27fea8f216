#!/bin/bash
# batch-1 decode A/B: short-context split attention partitions
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-300; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
for v in 0 64 0 64; do
  LOCALAI_AMD_DEC_SPLIT_SHORT=$v step q_c1_$v.log 300 python -u bench.py --mode engine --steps 3 --warmup 1 --concurrency 1 --max-tokens 256
done
