set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "moe or mixtral or qwen2moe or deepseek or router" > gpurun_out/pytest_moe.log 2>&1; rc=$?; grep -E "passed|failed|FAIL" gpurun_out/pytest_moe.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/mx_c1.log 2>&1; rc=$?; tail -1 gpurun_out/mx_c1.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 64 --max-tokens 128 > gpurun_out/mx_c64.log 2>&1; rc=$?; tail -1 gpurun_out/mx_c64.log | cut -c1-330; exit $rc
