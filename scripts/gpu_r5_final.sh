#!/bin/bash
# round-5 final: GPU test tier, smoke, and the headline bench twice, at HEAD
set -o pipefail
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r5_heartbeat.log; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r5_final2_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final2_smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r5_final2_bench.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r5_final2_bench2.log 2>&1
rc=$?
kill $HB
exit $rc
