# kernel-time check of act8 in the C=256 engine decode (compare act_kernel 6.4 us in profiles/engine_c256_v4.md)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 0 --concurrency 256 --max-tokens 64 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M (act8)" > $R/gpurun_out/prof_c256_act8.md && grep -E "act8_kernel|act_kernel|Decode steady|us wall" $R/gpurun_out/prof_c256_act8.md
