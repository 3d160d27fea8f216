set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5; exit $rc
