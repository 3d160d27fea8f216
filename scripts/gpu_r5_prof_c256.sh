#!/bin/bash
# Round 5: C=256 engine decode + prefill kernel tables (rocprofv3 kernel-trace/stats only)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/r5_prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M (round 5)" --steady 32 --by-grid 32 > $R/gpurun_out/r5_prof_c256.md && tail -5 $R/gpurun_out/r5_prof_c256.md
