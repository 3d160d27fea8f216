# GPU tests + engine/http benches + a decode profile.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 64 > gpurun_out/b_eng64.log 2>&1 && tail -1 gpurun_out/b_eng64.log &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_http256.log 2>&1 && tail -1 gpurun_out/b_http256.log &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 64 > $R/gpurun_out/prof_c1.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 0 --concurrency 256 --max-tokens 64 > $R/gpurun_out/prof_c256.log 2>&1 && echo PROF_OK
