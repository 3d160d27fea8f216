#!/bin/bash
# headline bench at the final HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_final3_bench.log 2>&1
