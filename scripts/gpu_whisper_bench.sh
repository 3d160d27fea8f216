set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python scripts/whisper_bench.py > gpurun_out/whisper_bench.log 2>&1; rc=$?; tail -1 gpurun_out/whisper_bench.log | cut -c1-300; exit $rc
