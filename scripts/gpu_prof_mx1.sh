# Kernel breakdown of Mixtral-8x7B decode at C=1 (engine).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 0 --concurrency 1 --max-tokens 4 > gpurun_out/mx_gen.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/mx1 -o run --output-format csv -- python3 $R/bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_mx1.log 2>&1 &&
python3 $R/scripts/prof_tail.py /tmp/la_prof/mx1 200 "Mixtral-8x7B Q4_K_M decode, C=1 (last 200 ms)" > $R/gpurun_out/prof_mx1.md && cat $R/gpurun_out/prof_mx1.md | head -30
