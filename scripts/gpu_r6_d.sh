export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_bs_gpu.py > gpurun_out/r6d_test.log 2>&1; tail -2 gpurun_out/r6d_test.log
timeout -k 10 400 python -u scripts/bs_bench.py --m 256 --shapes qkv,o,gate_up,down,lm_head > gpurun_out/r6d_b256.log 2>&1; cat gpurun_out/r6d_b256.log
timeout -k 10 300 python -u scripts/bs_bench.py --m 8192 --shapes gate_up,down6,qkv,o > gpurun_out/r6d_b8k.log 2>&1; cat gpurun_out/r6d_b8k.log
