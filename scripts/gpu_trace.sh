# Engine timeline of the C=256 and C=1 engine benches (host gaps between GPU work)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
LOCALAI_AMD_TRACE=/tmp/t256.json timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_t256.log 2>&1 && tail -1 gpurun_out/b_t256.log | cut -c1-160 && python scripts/trace_gaps.py /tmp/t256.json &&
LOCALAI_AMD_TRACE=/tmp/t1.json timeout -k 10 300 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_t1.log 2>&1 && tail -1 gpurun_out/b_t1.log | cut -c1-160 && python scripts/trace_gaps.py /tmp/t1.json
