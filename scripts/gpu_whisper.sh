set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_whisper.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_wh.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_wh.log | tail -8; exit $rc
