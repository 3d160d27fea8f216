set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
GEMV_SHAPES=q8 GEMV_VARIANTS=5,1,9,21 timeout -k 10 300 python scripts/gemv_variants.py > gpurun_out/q8v.log 2>&1; rc=$?; cat gpurun_out/q8v.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
GEMV_SHAPES=q8 GEMV_SWEEP_S=1 timeout -k 10 300 python scripts/gemv_variants.py > gpurun_out/q8s.log 2>&1; cat gpurun_out/q8s.log | grep -v amdgpu.ids
