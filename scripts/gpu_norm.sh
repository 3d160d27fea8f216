# add_norm numerics + C=1 engine decode + C=1 kernel profile summary
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "add_norm or rope" --timeout 120 --timeout-method thread > gpurun_out/pytest_norm.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_norm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-400 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c1 "Engine C=1, Llama-3-8B Q4_K_M" > $R/gpurun_out/prof_c1.md && sed -n '/Decode steady/,$p' $R/gpurun_out/prof_c1.md | head -12
