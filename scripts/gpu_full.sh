# Full check: all GPU tests, smoke, default bench (http C=256), engine C=1, profile C=256 + C=1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 600 python bench.py > gpurun_out/b_default.log 2>&1 && tail -1 gpurun_out/b_default.log | cut -c1-330 &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-200 &&
P=/tmp/la_prof && cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py $P/c256 "Engine C=256, Llama-3-8B Q4_K_M (warm-up wave + 1 timed wave)" > $R/gpurun_out/prof_c256.md &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py $P/c1 "Engine C=1, Llama-3-8B Q4_K_M (2 x 128 decode steps)" --decode-steps 256 > $R/gpurun_out/prof_c1.md && echo PROF_OK
