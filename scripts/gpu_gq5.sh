#!/bin/bash
# tile GEMM tests (incl. two-segment launch) + MoE any-batch tests, GEMM sweep, engine bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gemm_tile_gpu.py \
  "tests/test_kernels_gpu.py::test_moe_grouped_gemm" tests/test_kernels_gpu.py::test_moe_route_skewed_large \
  tests/test_kernels_gpu.py::test_moe_grouped_gemm_expert_parallel \
  tests/test_engine_gpu.py::test_mixtral_moe_graph_decode tests/test_engine_gpu.py::test_mixtral_moe_wide_batch_graph_decode \
  > gpurun_out/gq_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gq_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u scripts/gq_bench.py --m 256 128 --shapes qkv,o,gate_up,down,down6,lm_head > gpurun_out/gq_bench5.log 2>&1 || exit $?
cat gpurun_out/gq_bench5.log
timeout -k 10 420 python -u bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r3_bench_engine5.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_engine5.log
