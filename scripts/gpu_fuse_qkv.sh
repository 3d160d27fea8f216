# fused q|k|v GEMV + RoPE + KV append (batch-1/2 decode): GPU suite, C=1 / C=2 / C=256 engine benches, C=1 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-200 &&
LOCALAI_AMD_QKV_ROPE=0 timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1_unfused.log 2>&1 && tail -1 gpurun_out/b_eng1_unfused.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 2 --max-tokens 128 > gpurun_out/b_eng2.log 2>&1 && tail -1 gpurun_out/b_eng2.log | cut -c1-200 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/c1 -o run --output-format csv -- python3 $R/bench.py --mode engine --steps 1 --warmup 1 --concurrency 1 --max-tokens 128 > $R/gpurun_out/prof_c1.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/c1 "Engine C=1, Llama-3-8B Q4_K_M" --steady 32 --by-grid 32 > $R/gpurun_out/prof_c1.md && tail -40 $R/gpurun_out/prof_c1.md
