# Phi-2 Q4_K (BASELINE.json config 1's model; the reference runs it on llama.cpp's CPU backend) on one MI355X.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python bench.py --mode engine --preset phi2 --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/phi2_c1.log 2>&1; rc=$?; tail -1 gpurun_out/phi2_c1.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --preset phi2 --steps 2 --warmup 1 --concurrency 256 > gpurun_out/phi2_h256.log 2>&1; rc=$?; tail -1 gpurun_out/phi2_h256.log | cut -c1-330; exit $rc
