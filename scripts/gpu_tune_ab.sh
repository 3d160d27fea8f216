# C=256 engine bench: library-GEMM tuning (TunableOp) on vs off
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
LOCALAI_AMD_BLAS_TUNE=0 timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_tune0.log 2>&1 && tail -1 gpurun_out/b_tune0.log | cut -c1-200 && grep -o '"setup_s.*' gpurun_out/b_tune0.log &&
timeout -k 10 900 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_tune1.log 2>&1 && tail -1 gpurun_out/b_tune1.log | cut -c1-200 && grep -o '"setup_s.*' gpurun_out/b_tune1.log && ls -la /tmp/la_cache && wc -l /tmp/la_cache/*.csv && cp /tmp/la_cache/*.csv gpurun_out/ &&
timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_tune2.log 2>&1 && tail -1 gpurun_out/b_tune2.log | cut -c1-200 && grep -o '"setup_s.*' gpurun_out/b_tune2.log
