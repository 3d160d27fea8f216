# sampler argmax batching: sampling kernel tests + C=1 engine bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample" > gpurun_out/pytest_sample.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_sample.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-160
