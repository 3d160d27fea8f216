#!/bin/bash
# Tile GEMM (gemm_q.hip): numerics tests, then the shape sweep vs hipBLASLt + ablations.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gemm_tile_gpu.py > gpurun_out/gq_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gq_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u scripts/gq_bench.py --m 256 --shapes qkv,o,gate_up,down,lm_head --abl > gpurun_out/gq_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gq_bench.py --m 8192 --shapes qkv,o,gate_up,down --blas >> gpurun_out/gq_bench.log 2>&1
rc2=$?
cat gpurun_out/gq_bench.log
exit $rc2
