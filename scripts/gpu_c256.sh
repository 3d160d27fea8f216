# M=256 GEMM map (cold) + engine C=256 bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mid or linear or dequant" > gpurun_out/pytest_mid.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_mid.log; [ $rc -eq 0 ] || exit $rc
GEMM_MS=256 GEMM_SHAPES=qk,o,gate_up,down timeout -k 10 300 python scripts/gemm_map.py > gpurun_out/gemm256.log 2>&1 && grep -v amdgpu.ids gpurun_out/gemm256.log &&
timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency 256 > gpurun_out/b_eng256.log 2>&1 && tail -1 gpurun_out/b_eng256.log | cut -c1-400
