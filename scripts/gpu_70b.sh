# Llama-3-70B Q4_K_M (random-init) on ONE MI355X: C=1 and C=32 engine decode
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache70
mkdir -p $LOCALAI_AMD_CACHE
df -h /tmp | tail -1
avail=$(df --output=avail -k /tmp | tail -1)
[ "$avail" -gt 60000000 ] || { echo "not enough /tmp space: $avail KiB"; exit 3; }
free -g | head -2
timeout -k 10 1000 python -u bench.py --mode engine --preset llama3-70b --steps 1 --warmup 1 --concurrency 1 --max-tokens 64 --context 1024 > gpurun_out/b70_c1.log 2>&1; rc=$?; tail -3 gpurun_out/b70_c1.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --mode engine --preset llama3-70b --steps 1 --warmup 1 --concurrency 32 --max-tokens 64 --context 1024 > gpurun_out/b70_c32.log 2>&1; rc=$?; tail -1 gpurun_out/b70_c32.log | cut -c1-400; exit $rc
