#!/bin/bash
# grammar fix-up path: GPU equality test, mixed-batch decode, function calling C=32; FLUX GPU test
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LOCALAI_AMD_CACHE=/tmp/la_cache
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py::test_grammar_rows_fixed_up_beside_device_sampling tests/test_flux.py tests/test_sd3.py tests/test_sd.py::test_controlnet_on_gpu_graph -m gpu -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_gr.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s2_gr.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/mixed_batch_bench.py > gpurun_out/s2_mixed2.log 2>&1
rc=$?
grep "decode" gpurun_out/s2_mixed2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/fc_bench.py --concurrency 32 > gpurun_out/s2_fc32.log 2>&1; rc=$?; tail -1 gpurun_out/s2_fc32.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/lmhead_bmm_check.py > gpurun_out/s2_lmhead.log 2>&1; rc=$?; grep LMHEAD gpurun_out/s2_lmhead.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemv_sweep.py --preset 70b > gpurun_out/s2_gemv70b.md 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/s2_gemv70b.md; exit $rc
