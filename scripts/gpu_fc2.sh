# Function calling after the grammar trie / batched top-N change, then Mixtral C=64 (heartbeat on).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python scripts/fc_bench.py --concurrency 32 > gpurun_out/fc32.log 2>&1; rc=$?; tail -1 gpurun_out/fc32.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 64 --max-tokens 128 > gpurun_out/mx_c64.log 2>&1; rc=$?; tail -1 gpurun_out/mx_c64.log | cut -c1-400; exit $rc
