#!/bin/bash
# tile 2 (128x256, 2x4 waves) as a decode / GLU autotune candidate: numerics, choices, HTTP bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/t2_tests.log
[ $rc -eq 0 ] || exit $rc
BENCH_DUMP_GEMM=1 timeout -k 10 400 python -u bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 --max-tokens 256 > gpurun_out/t2_engine.log 2>&1
rc=$?; grep -E "glu choice M=2|choice M=256" gpurun_out/t2_engine.log | head -20; tail -1 gpurun_out/t2_engine.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 8 --warmup 2 > gpurun_out/t2_http.log 2>&1 && tail -1 gpurun_out/t2_http.log | cut -c1-200
