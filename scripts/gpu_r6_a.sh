set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_bs_gpu.py > gpurun_out/r6a_test.log 2>&1
rc=$?; tail -5 gpurun_out/r6a_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bs_bench.py --m 256 > gpurun_out/r6a_bench256.log 2>&1 && cat gpurun_out/r6a_bench256.log
timeout -k 10 300 python -u scripts/bs_bench.py --m 8192 --shapes gate_up,down,qkv,o > gpurun_out/r6a_bench8k.log 2>&1 ; cat gpurun_out/r6a_bench8k.log
