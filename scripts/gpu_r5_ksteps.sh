#!/bin/bash
# decode steps per host round trip: default (8 / 16 wide) vs 32
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_k_def.log 2>&1 || exit $?
BENCH_DECODE_STEPS=32 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k_32.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_k_def2.log 2>&1 || exit $?
BENCH_DECODE_STEPS=32 timeout -k 10 500 python -u bench.py > gpurun_out/r5_k_32b.log 2>&1
