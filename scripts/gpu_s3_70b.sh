# Llama-3-70B Q4_K_M (random-init) on ONE MI355X, C=1 engine decode (70B GEMV split tuning check)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache70
mkdir -p $LOCALAI_AMD_CACHE
avail=$(df --output=avail -k /tmp | tail -1)
[ "$avail" -gt 60000000 ] || { echo "not enough /tmp space: $avail KiB"; exit 3; }
( while true; do date >> gpurun_out/heartbeat70.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u bench.py --mode engine --preset llama3-70b --steps 1 --warmup 1 --concurrency 1 --max-tokens 64 --context 1024 > gpurun_out/s3_b70_c1.log 2>&1; rc=$?; tail -2 gpurun_out/s3_b70_c1.log | cut -c1-400; exit $rc
