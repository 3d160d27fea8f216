#!/bin/bash
# tile GEMM + GLU-fused tests, GEMM sweep (Q6_K dequant), engine bench with the tuned choices
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gemm_tile_gpu.py \
  > gpurun_out/gq_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gq_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u scripts/gq_bench.py --m 256 --shapes qkv,down,down6,lm_head > gpurun_out/gq_bench6.log 2>&1 || exit $?
cat gpurun_out/gq_bench6.log
BENCH_DUMP_GEMM=1 timeout -k 10 420 python -u bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r3_bench_engine6.log 2>&1 || exit $?
grep "glu choice" gpurun_out/r3_bench_engine6.log
tail -1 gpurun_out/r3_bench_engine6.log
