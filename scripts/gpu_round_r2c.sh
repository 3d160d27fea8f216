# Round-end rehearsal on HEAD (session 3): GPU suite (one process), smoke(), default bench line,
# engine C=256 and C=1 lines, and an HTTP C=256 kernel profile summary.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log | cut -c1-420 &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 > gpurun_out/bench_eng256.log 2>&1 && tail -1 gpurun_out/bench_eng256.log | cut -c1-420 &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/bench_eng1.log 2>&1 && tail -1 gpurun_out/bench_eng1.log | cut -c1-420 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/h256 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --concurrency 256 --max-tokens 128 > $R/gpurun_out/prof_h256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/h256 "HTTP C=256, Llama-3-8B Q4_K_M (round-2 session-3 HEAD)" > $R/gpurun_out/prof_h256.md && echo PROF_OK
