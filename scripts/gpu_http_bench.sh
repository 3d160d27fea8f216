# HTTP-mode bench (the headline metric) on the native server; uvicorn + engine-mode comparisons.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_http.log 2>&1 && echo BENCH_HTTP_OK && tail -1 gpurun_out/bench_http.log &&
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --concurrency 256 > gpurun_out/bench_http256.log 2>&1 && echo BENCH_HTTP256_OK && tail -1 gpurun_out/bench_http256.log &&
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --concurrency 256 --mode engine > gpurun_out/bench_eng256.log 2>&1 && echo BENCH_ENG256_OK && tail -1 gpurun_out/bench_eng256.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/bench_http1.log 2>&1 && echo BENCH_HTTP1_OK && tail -1 gpurun_out/bench_http1.log
