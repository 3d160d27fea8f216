set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
GEMV_SWEEP_S=1 timeout -k 10 500 python -u scripts/gemv_variants.py > gpurun_out/gemv_sweep_s.log 2>&1 && cat gpurun_out/gemv_sweep_s.log &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or linear_multi or act_linear" > gpurun_out/pytest_dp4.log 2>&1 && tail -1 gpurun_out/pytest_dp4.log &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-200
