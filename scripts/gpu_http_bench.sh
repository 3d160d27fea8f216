# HTTP-mode bench (the headline metric) + engine-mode comparison + GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_http.log 2>&1 && echo BENCH_HTTP_OK && tail -1 gpurun_out/bench_http.log &&
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --concurrency 256 > gpurun_out/bench_http256.log 2>&1 && echo BENCH_HTTP256_OK && tail -1 gpurun_out/bench_http256.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/bench_http1.log 2>&1 && echo BENCH_HTTP1_OK && tail -1 gpurun_out/bench_http1.log
