set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 128 > gpurun_out/bench_engine128.log 2>&1 && echo B128 && tail -1 gpurun_out/bench_engine128.log &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/bench_engine256.log 2>&1 && echo B256 && tail -1 gpurun_out/bench_engine256.log &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/bench_engine1.log 2>&1 && echo B1 && tail -1 gpurun_out/bench_engine1.log &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof64 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 0 --concurrency 64 --max-tokens 64 > $R/gpurun_out/prof64.log 2>&1 && echo PROF_OK
