# gemm_dq bring-up: numerics tests, ablation probe, then cold-cache timings at the decode shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dq_gemm" > gpurun_out/pytest_dq.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_dq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dq_probe.py > gpurun_out/dq_probe.log 2>&1; rc=$?; cat gpurun_out/dq_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dq_bench.py 256 > gpurun_out/dq_bench.log 2>&1; rc=$?; cat gpurun_out/dq_bench.log; exit $rc
