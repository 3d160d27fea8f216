set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or linear_multi" > gpurun_out/pytest_dp4.log 2>&1 && tail -2 gpurun_out/pytest_dp4.log &&
timeout -k 10 400 python -u scripts/gemv_variants.py > gpurun_out/gemv_variants.log 2>&1 && cat gpurun_out/gemv_variants.log
