# round-2 HEAD profiles: C=256 and C=1 engine decode (per kernel, per (kernel, grid)), plus both bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M (round-2 HEAD)" --steady 32 --by-grid 32 > $R/gpurun_out/prof_c256.md &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c1 "Engine C=1, Llama-3-8B Q4_K_M (round-2 HEAD)" --steady 32 --by-grid 32 > $R/gpurun_out/prof_c1.md &&
grep -A3 "Decode steady" $R/gpurun_out/prof_c256.md && grep -A3 "Decode steady" $R/gpurun_out/prof_c1.md
