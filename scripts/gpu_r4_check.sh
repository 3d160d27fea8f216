#!/bin/bash
# round-4 GPU check: custom all-reduce at world 2/4/8 (ranks sharing the GPU), TP + engine GPU
# tests, then the driver's default bench and the gateway-mode bench shape at N=1.
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
run() { local n=$1; shift; timeout -k 10 "$@" > gpurun_out/$LOG 2>&1; rc=$?; tail -4 gpurun_out/$LOG; [ $rc -eq 0 ] || { tail -40 gpurun_out/$LOG; exit $rc; }; }
LOG=t_ar.log run 0 600 python -u -m pytest tests/test_custom_allreduce.py tests/test_tp_gpu.py -x -v --timeout 300 --timeout-method thread
LOG=t_eng.log run 0 900 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_tile_gpu.py -x -q --timeout 300 --timeout-method thread
LOG=b_http.log run 0 600 python -u bench.py
