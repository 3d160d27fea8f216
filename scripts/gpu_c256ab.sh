# C=256 / C=512 engine benches (+ GEMM path choices) and a C=256 steady-state profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
BENCH_DUMP_GEMM=1 timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log | cut -c1-200 && grep "gemm choice M=256\|gemm choice M=128" gpurun_out/b_eng256.log | cut -c1-200 &&
timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 512 > gpurun_out/b_eng512.log 2>&1 && tail -1 gpurun_out/b_eng512.log | cut -c1-400
