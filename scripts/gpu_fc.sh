# Function-calling throughput on MI355X (forced tool, GBNF-constrained sampling), C=32 and C=1.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 500 python scripts/fc_bench.py --concurrency 32 > gpurun_out/fc32.log 2>&1; rc=$?; tail -1 gpurun_out/fc32.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fc_bench.py --concurrency 1 --waves 3 > gpurun_out/fc1.log 2>&1; rc=$?; tail -1 gpurun_out/fc1.log | cut -c1-500; exit $rc
