#!/bin/bash
# tile GEMM v2 (pipelined schedules): numerics, decode-shape sweep, then counters
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gemm_tile_gpu.py > gpurun_out/gq_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gq_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u scripts/gq_bench.py --m 256 128 --shapes qkv,o,gate_up,down,down6,lm_head --abl > gpurun_out/gq_bench2.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gq_bench.py --m 8192 --shapes qkv,gate_up,down >> gpurun_out/gq_bench2.log 2>&1 || exit $?
cat gpurun_out/gq_bench2.log
bash scripts/gpu_gq_pmc.sh
