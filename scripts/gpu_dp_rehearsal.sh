# Rehearse the driver's multi-rank bench launch (2 ranks sharing the one GPU over gloo).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 64 --max-tokens 64 > gpurun_out/b_dp2.log 2>&1; rc=$?; tail -3 gpurun_out/b_dp2.log | cut -c1-400; exit $rc
