set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemv_mall_probe.py > gpurun_out/mall_probe.log 2>&1; rc=$?; cat gpurun_out/mall_probe.log; exit $rc
