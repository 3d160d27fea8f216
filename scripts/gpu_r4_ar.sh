#!/bin/bash
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_custom_allreduce.py tests/test_tp_gpu.py > gpurun_out/ar_final.log 2>&1; rc=$?
grep -E "passed|failed|retrying" gpurun_out/ar_final.log | tail -5
exit $rc
