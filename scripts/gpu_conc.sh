# Throughput vs concurrency (engine and HTTP) on Llama-3-8B Q4_K_M.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
for C in 384 512; do
  timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency $C > gpurun_out/b_eng$C.log 2>&1 || exit 1
  tail -1 gpurun_out/b_eng$C.log | cut -c1-420
done
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --concurrency 512 > gpurun_out/b_http512.log 2>&1 && tail -1 gpurun_out/b_http512.log | cut -c1-420
