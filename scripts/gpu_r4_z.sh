#!/bin/bash
# function calling C=32: constrained-majority batches single-step (default) vs riding multi-step runs
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; grep -h "metric" gpurun_out/$log | cut -c1-260; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
step z_fc_def.log 400 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32 --max-tokens 128
LOCALAI_AMD_GRAMMAR_MIXED_FRAC=1.0 step z_fc_f1.log 400 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32 --max-tokens 128
LOCALAI_AMD_GRAMMAR_MIXED_FRAC=1.0 LOCALAI_AMD_GRAMMAR_MIXED_K=8 step z_fc_f1k8.log 400 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32 --max-tokens 128
step z_fc_def2.log 400 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32 --max-tokens 128
LOCALAI_AMD_GRAMMAR_MIXED_FRAC=1.0 step z_fc_f1b.log 400 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32 --max-tokens 128
