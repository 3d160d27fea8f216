# round-3 session 2: int8-epilogue probe + GPU tests of the new features (draft model, TP overlap)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -Wno-unused-value -Wno-unused-result scripts/i8_epilogue_probe.hip -o /tmp/i8probe &&
timeout -k 10 120 /tmp/i8probe > gpurun_out/i8probe.log 2>&1 && cat gpurun_out/i8probe.log &&
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_engine_gpu.py::test_draft_model_speculation_on_gpu tests/test_tp_gpu.py tests/test_sdxl.py > gpurun_out/s2_tests.log 2>&1;
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s2_tests.log | tail -8; exit $rc
