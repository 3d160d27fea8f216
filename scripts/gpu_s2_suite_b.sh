#!/bin/bash
# resume the GPU suite from test_sdxl onward (+ the SD file for the ControlNet GPU test), then smoke
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sd.py tests/test_sdxl.py tests/test_spec_prompt_cache.py tests/test_sysinfo.py tests/test_templates.py tests/test_tp_gloo.py tests/test_tp_gpu.py tests/test_tts.py tests/test_whisper.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_suite_b.log 2>&1
rc=$?
tail -4 gpurun_out/s2_suite_b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke.log 2>&1
rc=$?
tail -2 gpurun_out/s2_smoke.log
exit $rc
