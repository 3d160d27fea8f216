set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python scripts/mid_probe.py > gpurun_out/mid_probe.log 2>&1; rc=$?; cat gpurun_out/mid_probe.log | grep -v amdgpu.ids; exit $rc
