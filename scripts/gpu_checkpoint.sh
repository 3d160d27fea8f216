# GPU suite + smoke + default bench (the driver's round-end sequence) on the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash scripts/gpu_suite.sh && 
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log
