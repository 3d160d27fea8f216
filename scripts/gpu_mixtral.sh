# Mixtral-8x7B Q4_K_M (random-init) on one MI355X: engine decode throughput at C=1 and C=64
# (BASELINE.json config 4: MoE expert-routed dequant GEMM).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 500 python bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/mx_c1.log 2>&1; rc=$?; tail -1 gpurun_out/mx_c1.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 64 --max-tokens 128 > gpurun_out/mx_c64.log 2>&1; rc=$?; tail -1 gpurun_out/mx_c64.log | cut -c1-330; exit $rc
