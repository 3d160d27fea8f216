# ws GEMM bring-up: numerics, then M=256 map
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 60 --timeout-method thread -k "ws_gemm or mid" > gpurun_out/pytest_ws.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_ws.log; [ $rc -eq 0 ] || exit $rc
GEMM_MS=256 GEMM_SHAPES=qk,o,gate_up,down timeout -k 10 300 python scripts/gemm_map.py > gpurun_out/gemm256.log 2>&1; grep -v amdgpu.ids gpurun_out/gemm256.log | sort -k1,1 -k5,5n | awk '{k=$1; if (c[k]++ < 5) print}'
