#!/bin/bash
# engine-mode and HTTP headline bench (tile GEMM path)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_DUMP_GEMM=1 timeout -k 10 420 python -u bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r3_bench_engine5.log 2>&1 || { tail -20 gpurun_out/r3_bench_engine5.log; exit 3; }
tail -1 gpurun_out/r3_bench_engine5.log; grep "M=256" gpurun_out/r3_bench_engine5.log
