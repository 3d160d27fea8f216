set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 360 --timeout-method thread > gpurun_out/pytest_tp.log 2>&1; rc=$?; grep -E "PASS|FAIL|TP |Error|assert" gpurun_out/pytest_tp.log | tail -12; exit $rc
