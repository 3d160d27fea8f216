# dp4 decode GEMV: numerics + per-shape timing against the skinny MFMA kernel (cold weights)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or skinny or linear_multi or mid_gemm" > gpurun_out/pytest_dp4.log 2>&1 && tail -3 gpurun_out/pytest_dp4.log &&
GEMM_MS=${GEMM_MS:-1,2,4} timeout -k 10 400 python -u scripts/gemm_map.py > gpurun_out/gemv_dp4_map.log 2>&1 && cat gpurun_out/gemv_dp4_map.log
