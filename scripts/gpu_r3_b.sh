#!/bin/bash
# new GPU tests (headline numerics vs fp32 oracle, audio models on device, smoke) + batch-1 decode bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_engine_gpu.py::test_headline_path_against_fp32_oracle tests/test_tts.py tests/test_audio_gen.py -m gpu \
  > gpurun_out/r3b_tests.log 2>&1
rc=$?
grep -E "headline numerics|passed|failed|Error" gpurun_out/r3b_tests.log | tail -8
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; tail -40 gpurun_out/r3b_tests.log; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.log 2>&1 || { tail -20 gpurun_out/r3b_smoke.log; exit 1; }
tail -1 gpurun_out/r3b_smoke.log
timeout -k 10 400 python -u bench.py --mode engine --concurrency 1 --max-tokens 256 --steps 2 --warmup 1 > gpurun_out/r3b_c1.log 2>&1 || exit $?
tail -1 gpurun_out/r3b_c1.log
