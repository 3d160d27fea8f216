#!/bin/bash
# decode-attention variants (numerics + timing), SD-family fp32 checks, mixed grammar batches,
# Mixtral function calling with room for the whole call
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
for v in 0 1 2 3; do
  LOCALAI_AMD_ATTN_VAR=$v step t_attn$v.log 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attn_decode
  LOCALAI_AMD_ATTN_VAR=$v step attn_b$v.log 200 python -u scripts/attn_bench.py
  grep "B=256\|B=128\|B=512" gpurun_out/attn_b$v.log
done
step t_fp32.log 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_sd.py tests/test_sdxl.py tests/test_flux.py tests/test_sd3.py -k "fp32_forward or graph_matches_eager"
grep -h "denoiser vs" gpurun_out/t_fp32.log
step t_mixed.log 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "rides"
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
step fc_mx.log 800 python -u scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32 --max-tokens 128
