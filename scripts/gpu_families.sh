set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "attn or families" > gpurun_out/pytest_fam.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_fam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 256 > gpurun_out/b_c1_base.log 2>&1 && tail -1 gpurun_out/b_c1_base.log | cut -c1-180 &&
timeout -k 10 400 python scripts/norm_ub.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 256 > gpurun_out/b_c1_ub.log 2>&1 && tail -1 gpurun_out/b_c1_ub.log | cut -c1-180
