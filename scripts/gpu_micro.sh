set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python scripts/microbench.py --out gpurun_out/micro.json > gpurun_out/micro.log 2>&1; tail -60 gpurun_out/micro.log
