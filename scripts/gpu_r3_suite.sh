#!/bin/bash
# Round-3 checkpoint: full GPU suite, then engine-mode and HTTP headline bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r3_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 420 python -u bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/r3_bench_engine.log 2>&1 || { echo "engine bench failed"; tail -20 gpurun_out/r3_bench_engine.log; exit 3; }
tail -2 gpurun_out/r3_bench_engine.log
timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r3_bench_http.log 2>&1
rc3=$?
tail -2 gpurun_out/r3_bench_http.log
exit $rc3
