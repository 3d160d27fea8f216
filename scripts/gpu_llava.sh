set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python scripts/llava_bench.py --concurrency 1 --waves 2 > gpurun_out/llava1.log 2>&1; rc=$?; tail -1 gpurun_out/llava1.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/llava_bench.py --concurrency 16 > gpurun_out/llava16.log 2>&1; rc=$?; tail -1 gpurun_out/llava16.log | cut -c1-400; exit $rc
