# C=256: HTTP (bench default) vs engine, engine timeline gaps, steady-state kernel profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/b_http256.log 2>&1 && tail -1 gpurun_out/b_http256.log | cut -c1-330 &&
LOCALAI_AMD_TRACE=/tmp/th.json timeout -k 10 600 python bench.py --steps 1 --warmup 1 > gpurun_out/b_http256t.log 2>&1 && python scripts/trace_gaps.py /tmp/th.json &&
LOCALAI_AMD_TRACE=/tmp/te.json timeout -k 10 600 python bench.py --mode engine --steps 1 --warmup 1 > gpurun_out/b_eng256t.log 2>&1 && python scripts/trace_gaps.py /tmp/te.json &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M" --steady 32 > $R/gpurun_out/prof_c256.md && tail -24 $R/gpurun_out/prof_c256.md
