#!/bin/bash
# HTTP vs engine mode after the native fast route (same box, alternated)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r5_he2_http.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --mode engine > gpurun_out/r5_he2_engine.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r5_he2_http2.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gateway_profile.py > gpurun_out/r5_he2_gwprof.log 2>&1
