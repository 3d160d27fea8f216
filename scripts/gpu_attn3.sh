set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn" > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_e256_nw1.log 2>&1 && tail -1 gpurun_out/b_e256_nw1.log | cut -c1-200 &&
LOCALAI_AMD_DEC_NW1_MIN=1000000 timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_e256_nw4.log 2>&1 && tail -1 gpurun_out/b_e256_nw4.log | cut -c1-200
