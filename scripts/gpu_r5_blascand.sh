#!/bin/bash
# decode GEMM autotune with hipBLASLt on the resident bf16 copies as a candidate
set -o pipefail
mkdir -p gpurun_out
LOCALAI_AMD_BLAS_CANDIDATE=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_blascand_on.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_blascand_off.log 2>&1 || exit $?
LOCALAI_AMD_BLAS_CANDIDATE=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_blascand_on2.log 2>&1
