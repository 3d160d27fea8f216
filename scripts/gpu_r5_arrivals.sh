#!/bin/bash
# server-side arrival spread and admission window of the HTTP burst
set -o pipefail
mkdir -p gpurun_out
BENCH_ARRIVALS=1 timeout -k 10 500 python -u bench.py > gpurun_out/r5_arr_http.log 2>&1 || exit $?
BENCH_ARRIVALS=1 timeout -k 10 500 python -u bench.py --mode engine > gpurun_out/r5_arr_engine.log 2>&1
