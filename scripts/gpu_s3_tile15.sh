#!/bin/bash
# 4-wave 128x256 tile (id 15): numerics, autotune choices at the C=256 shapes, HTTP A/B vs without it
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_tile_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t15_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t15_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_DUMP_GEMM=1 timeout -k 10 400 python -u bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 --max-tokens 256 > gpurun_out/t15_engine.log 2>&1
rc=$?; grep -E "glu choice|choice M=2[0-9][0-9]" gpurun_out/t15_engine.log | head -30; tail -1 gpurun_out/t15_engine.log | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 8 --warmup 2 > gpurun_out/t15_http.log 2>&1 && tail -1 gpurun_out/t15_http.log | cut -c1-250
