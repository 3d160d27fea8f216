#!/bin/bash
# prefill chunk budget (max_batched_tokens) A/B under burst prefill-first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_ch_8k.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --batch-tokens 16384 > gpurun_out/r5_ch_16k.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --batch-tokens 12288 > gpurun_out/r5_ch_12k.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_ch_8k2.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --batch-tokens 16384 > gpurun_out/r5_ch_16k2.log 2>&1
