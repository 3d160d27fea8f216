set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 900 python scripts/gemm_tune_probe.py > gpurun_out/gemm_tune_probe.log 2>&1; rc=$?; tail -30 gpurun_out/gemm_tune_probe.log; exit $rc
