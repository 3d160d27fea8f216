# prefill-dominated waves (256 prompts x 128 tokens, 2 generated): kernel breakdown of the last wave
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/pf -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 --max-tokens 2 > $R/gpurun_out/prof_pf.log 2>&1 &&
tail -1 $R/gpurun_out/prof_pf.log | cut -c1-250 &&
python3 $R/scripts/prof_tail.py /tmp/la_prof/pf 700 "Prefill wave: 256 prompts x ~140 tokens, Llama-3-8B Q4_K_M" > $R/gpurun_out/prof_pf.md && cat $R/gpurun_out/prof_pf.md
