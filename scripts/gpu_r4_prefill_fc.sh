#!/bin/bash
# prefill-size GEMMs (library vs hand-written) + Mixtral-8x7B function calling at C=32
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u scripts/prefill_gemm_bench.py --m 2048 8192 --check > gpurun_out/pf_gemm.log 2>&1; rc=$?; cat gpurun_out/pf_gemm.log | grep -v "^check" | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32 > gpurun_out/fc_mx32.log 2>&1; rc=$?; tail -2 gpurun_out/fc_mx32.log | cut -c1-700; exit $rc
