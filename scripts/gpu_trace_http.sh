# Engine timeline under the HTTP bench vs the in-process engine bench (C=256): step durations and host gaps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
LOCALAI_AMD_TRACE=/tmp/th.json timeout -k 10 600 python bench.py --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_th.log 2>&1 && tail -1 gpurun_out/b_th.log | cut -c1-200 && python scripts/trace_gaps.py /tmp/th.json &&
LOCALAI_AMD_TRACE=/tmp/te.json timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > gpurun_out/b_te.log 2>&1 && tail -1 gpurun_out/b_te.log | cut -c1-200 && python scripts/trace_gaps.py /tmp/te.json
