# Round-3 session-2 baseline on HEAD: HTTP headline bench, then an engine C=256 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > gpurun_out/s2_http.log 2>&1 && tail -1 gpurun_out/s2_http.log | cut -c1-400 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/s2_prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M" --steady 32 > $R/gpurun_out/s2_prof_c256.md && tail -1 $R/gpurun_out/s2_prof_c256.log | cut -c1-300
