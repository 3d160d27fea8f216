#!/bin/bash
# resume the GPU suite from the SD tests onward (the earlier files passed in the previous call)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sd.py tests/test_spec_prompt_cache.py tests/test_sysinfo.py tests/test_templates.py tests/test_tp_gloo.py tests/test_tp_gpu.py tests/test_tts.py tests/test_whisper.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite2.log 2>&1
rc=$?
tail -5 gpurun_out/r3_suite2.log
exit $rc
