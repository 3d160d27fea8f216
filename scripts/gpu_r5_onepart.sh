#!/bin/bash
# batch-1/2 decode attention: single-partition threshold (no split-KV merge) 256 (default) vs 512 / 1024 keys
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn_decode" > gpurun_out/r5_op_tests.log 2>&1 || exit $?
LOCALAI_AMD_DEC_ONE_PART=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn_decode" >> gpurun_out/r5_op_tests.log 2>&1 || exit $?
B="python -u bench.py --mode engine --steps 3 --warmup 1 --max-tokens 256"
for C in 1 2; do
  timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_op_c${C}_256.log 2>&1 || exit $?
  LOCALAI_AMD_DEC_ONE_PART=512 timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_op_c${C}_512.log 2>&1 || exit $?
  LOCALAI_AMD_DEC_ONE_PART=1024 timeout -k 10 400 $B --concurrency $C > gpurun_out/r5_op_c${C}_1024.log 2>&1 || exit $?
done
