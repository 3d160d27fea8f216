# mid-M GEMM bring-up: kernel tests, then the GEMM microbench only.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q > gpurun_out/pytest_mid.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_mid.log; [ $rc -eq 0 ] || exit $rc
MB_ONLY_GEMM=1 timeout -k 10 600 python scripts/microbench.py --out gpurun_out/micro_mid.json > gpurun_out/micro_mid.log 2>&1; rc=$?; grep -E "^mid|^hipblas" gpurun_out/micro_mid.log; exit $rc
