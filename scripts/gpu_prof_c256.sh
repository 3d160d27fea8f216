# C=256 engine decode profile (per kernel and per (kernel, grid)), plus the default HTTP bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log | cut -c1-400 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M" --steady 32 --by-grid 32 > $R/gpurun_out/prof_c256.md && tail -45 $R/gpurun_out/prof_c256.md
