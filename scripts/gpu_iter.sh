# Iteration loop: GPU tests -> op microbench -> engine benches (C=1, 64, 256) -> http C=256.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/microbench.py --out gpurun_out/micro.json > gpurun_out/micro.log 2>&1; rc=$?; grep -E "attn|T=|M=  1 " gpurun_out/micro.log; [ $rc -eq 0 ] || exit $rc
for C in 1 64 256; do
  timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency $C > gpurun_out/b_eng$C.log 2>&1 || exit 1
  tail -1 gpurun_out/b_eng$C.log | cut -c1-330
done
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_http256.log 2>&1 && tail -1 gpurun_out/b_http256.log | cut -c1-330
