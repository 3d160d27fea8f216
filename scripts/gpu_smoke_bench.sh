set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 64 > gpurun_out/bench_engine64.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench_engine64.log
