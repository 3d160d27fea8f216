set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/rope_bench.py > gpurun_out/rope_bench.log 2>&1; rc=$?; cat gpurun_out/rope_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log; exit $rc
