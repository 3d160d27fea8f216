set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "families or lora or attn_decode or attn_prefill" > gpurun_out/pytest_fam.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/pytest_fam.log | tail -9; tail -2 gpurun_out/pytest_fam.log; exit $rc
