#!/bin/bash
# round-3 engine C=256 decode profile (per kernel, per (kernel, grid)) with the tile GEMM
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp &&
BENCH_DUMP_GEMM=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/prof_r3_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M (round-3 tile GEMM)" --steady 32 --by-grid 32 > $R/gpurun_out/prof_r3_c256.md &&
grep -A30 "Decode steady" $R/gpurun_out/prof_r3_c256.md && grep "gemm choice" $R/gpurun_out/prof_r3_c256.log | head -40
