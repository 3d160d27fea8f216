#!/bin/bash
# fused add_norm + MoE router: kernel test, MoE model GPU tests, Mixtral C=1 / C=256 A/B
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "add_norm_router" > gpurun_out/r5_nr_kern.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "moe or mixtral or qwen2moe or tp" > gpurun_out/r5_nr_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_nr_c1.log 2>&1 &&
LOCALAI_AMD_NORM_ROUTER=0 timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_nr_c1_off.log 2>&1 &&
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_nr_c1b.log 2>&1 &&
timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_nr_http.log 2>&1 &&
LOCALAI_AMD_NORM_ROUTER=0 timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5_nr_http_off.log 2>&1
rc=$?
kill $HB
exit $rc
