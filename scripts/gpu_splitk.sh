set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 240 python scripts/splitk_probe.py > gpurun_out/splitk.log 2>&1; rc=$?; cat gpurun_out/splitk.log | grep -v Warning; [ $rc -eq 0 ] || exit $rc
PROBE_TUNE=1 timeout -k 10 400 python scripts/splitk_probe.py > gpurun_out/splitk_tuned.log 2>&1; rc=$?; grep -v Warning gpurun_out/splitk_tuned.log; exit $rc
