set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache_15
timeout -k 10 900 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/b_base.log 2>&1 && echo "base: $(tail -1 gpurun_out/b_base.log | cut -c80-160)" || exit 1
LOCALAI_AMD_FUSED_ROPE=1 timeout -k 10 900 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/b_frope.log 2>&1 && echo "fused rope: $(tail -1 gpurun_out/b_frope.log | cut -c80-160)" || exit 1
export LOCALAI_AMD_CACHE=/tmp/la_cache_100
LOCALAI_AMD_BLAS_TUNE_MS=100 timeout -k 10 900 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/b_tune100.log 2>&1 && echo "tune 100 ms: $(tail -1 gpurun_out/b_tune100.log | cut -c80-160)"
