#!/bin/bash
# HTTP (default) vs engine mode TTFT on the same box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_he_http.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --mode engine > gpurun_out/r5_he_engine.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_he_http2.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --mode engine > gpurun_out/r5_he_engine2.log 2>&1
