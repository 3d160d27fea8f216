#!/bin/bash
# default build with MoE GEMV variant 1: MoE / Mixtral GPU tests, smoke, Mixtral C=1
set -o pipefail
mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "moe or mixtral or qwen2moe" > gpurun_out/r5_mv3_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_mv3_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/r5_mv3_c1.log 2>&1
rc=$?
kill $HB
exit $rc
