#!/bin/bash
# two-shot all-reduce: exactness (two ranks sharing the GPU), latency, TP engine rehearsal
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce.py tests/test_tp_gpu.py -m gpu -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_ar2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s2_ar2.log | tail -6
[ $rc -eq 0 ] || exit $rc
LOCALAI_AMD_AR_SAME_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 scripts/ar_check.py > gpurun_out/s2_ar2_check.log 2>&1
rc=$?
grep AR_OK gpurun_out/s2_ar2_check.log
exit $rc
