# fused bf16 q|k+v library GEMM: kernel test, C=256 engine bench, C=256 steady-state profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused_bf16 or linear" > gpurun_out/pytest_fuse.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_fuse.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log | cut -c1-200 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c256 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 256 --max-tokens 256 > $R/gpurun_out/prof_c256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c256 "Engine C=256, Llama-3-8B Q4_K_M" --steady 32 > $R/gpurun_out/prof_c256.md && grep -A16 "steady state" $R/gpurun_out/prof_c256.md
