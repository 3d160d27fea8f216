set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
LOCALAI_AMD_AR_SAME_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/ar_check.py > gpurun_out/ar_check.log 2>&1; rc=$?; tail -20 gpurun_out/ar_check.log; exit $rc
