#!/bin/bash
# q32 Q4_K dequant through v_cvt_pk_f32_fp8 (default build) vs v_cvt_f32_ubyte (LA_Q32_FP8=0 build)
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_tile_gpu.py tests/test_moe32_gpu.py > gpurun_out/r5_fp8_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/moe_bench.py --T 256 --vars 4 > gpurun_out/r5_fp8_moe.log 2>&1 || exit $?
LOCALAI_AMD_KLIB=_la_kernels_nofp8.so timeout -k 10 300 python -u scripts/moe_bench.py --T 256 --vars 4 > gpurun_out/r5_fp8_moe_off.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gq_bench.py --m 256 --shapes gate_up,down,qkv,o > gpurun_out/r5_fp8_gq.log 2>&1 || exit $?
LOCALAI_AMD_KLIB=_la_kernels_nofp8.so timeout -k 10 300 python -u scripts/gq_bench.py --m 256 --shapes gate_up,down,qkv,o > gpurun_out/r5_fp8_gq_off.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_fp8_bench.log 2>&1 || exit $?
LOCALAI_AMD_KLIB=_la_kernels_nofp8.so timeout -k 10 500 python -u bench.py > gpurun_out/r5_fp8_bench_off.log 2>&1
