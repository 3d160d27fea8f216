set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
LOCALAI_AMD_TRACE=/tmp/tw.json timeout -k 10 900 python bench.py > gpurun_out/b_unique.log 2>&1 && tail -1 gpurun_out/b_unique.log | cut -c1-330 && python scripts/trace_waves.py /tmp/tw.json
