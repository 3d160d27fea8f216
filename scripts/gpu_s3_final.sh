# Round-3 session-3 rehearsal on HEAD: smoke(), the driver's bench command, an engine C=256 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 && tail -2 gpurun_out/s3_smoke.log &&
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s3_bench.log 2>&1 && tail -1 gpurun_out/s3_bench.log | cut -c1-500 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/s3_prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M (round 3 session 3 HEAD)" --steady 32 > $R/gpurun_out/s3_prof_c256.md && tail -1 $R/gpurun_out/s3_prof_c256.log | cut -c1-300
