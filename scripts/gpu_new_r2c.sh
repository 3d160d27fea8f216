set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u -m pytest tests/test_mamba.py tests/test_hf_checkpoint.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; grep -E "passed|failed|error|PASS|FAIL" gpurun_out/pytest_new.log | tail -6; exit $rc
