# grouped-transposed V pages + rope_kv8: numerics, micro timings, engine C=1 / C=256
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/rope_bench.py > gpurun_out/rope_bench.log 2>&1 && cat gpurun_out/rope_bench.log &&
timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1 && cat gpurun_out/attn_bench.log &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-200 &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log | cut -c1-260
