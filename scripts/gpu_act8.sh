# act8 (16-byte vector SwiGLU/GELU) numerics + engine C=256 decode throughput
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "act" --timeout 120 --timeout-method thread > gpurun_out/pytest_act.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_act.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 --max-tokens 128 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log | cut -c1-300 &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 1 --max-tokens 128 > gpurun_out/b_eng1.log 2>&1 && tail -1 gpurun_out/b_eng1.log | cut -c1-300
