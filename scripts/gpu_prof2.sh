# rocprofv3 kernel profiles of the engine bench at C=1 and C=256 (summaries -> gpurun_out/*.md)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
P=/tmp/la_prof
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py $P/c1 "Engine C=1, Llama-3-8B Q4_K_M" > $R/gpurun_out/prof_c1.md &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py $P/c256 "Engine C=256, Llama-3-8B Q4_K_M" > $R/gpurun_out/prof_c256.md && echo PROF_OK
