set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
GEMV_VARIANTS=1,5,9 timeout -k 10 500 python -u scripts/gemv_variants.py > gpurun_out/gemv_rs.log 2>&1 && cat gpurun_out/gemv_rs.log
