set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
GEMV_SWEEP_S=1 timeout -k 10 300 python scripts/gemv_variants.py > gpurun_out/q4s.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/q4s.log; exit $rc
