# A/B: gemm_dq (in-register-dequant Q4_K GEMM) as an autotune candidate at decode batch 256.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache BENCH_DUMP_GEMM=1
timeout -k 10 400 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/dqab_base1.log 2>&1 && tail -1 gpurun_out/dqab_base1.log | cut -c1-330 &&
LOCALAI_AMD_DQ=1 timeout -k 10 400 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/dqab_dq.log 2>&1 && tail -1 gpurun_out/dqab_dq.log | cut -c1-330 &&
timeout -k 10 400 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/dqab_base2.log 2>&1 && tail -1 gpurun_out/dqab_base2.log | cut -c1-330 &&
grep "gemm choice M=256" gpurun_out/dqab_base1.log gpurun_out/dqab_dq.log
