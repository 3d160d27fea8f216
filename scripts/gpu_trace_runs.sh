set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
LOCALAI_AMD_TRACE=/tmp/tw.json timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/b_tr.log 2>&1 && tail -1 gpurun_out/b_tr.log | cut -c1-300 && python scripts/trace_runs.py /tmp/tw.json &&
LOCALAI_AMD_TRACE=/tmp/te.json timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/b_te.log 2>&1 && tail -1 gpurun_out/b_te.log | cut -c1-300 && python scripts/trace_runs.py /tmp/te.json
