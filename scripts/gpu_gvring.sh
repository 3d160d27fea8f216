# dp4 GEMV: default variant (5) vs the 4-deep weight ring everywhere it applies (21), C=1 / C=2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dp4 or act_linear" > gpurun_out/pytest_gv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gv.log; [ $rc -eq 0 ] || exit $rc
LOCALAI_AMD_GEMV_VARIANT=21 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dp4 or act_linear" > gpurun_out/pytest_gv21.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gv21.log; [ $rc -eq 0 ] || exit $rc
for v in 5 21; do
  for c in 1 2; do
    LOCALAI_AMD_GEMV_VARIANT=$v timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency $c --max-tokens 128 > gpurun_out/b_gv${v}_c$c.log 2>&1 || exit 1
    echo "variant $v C=$c: $(tail -1 gpurun_out/b_gv${v}_c$c.log | cut -c100-130)"
  done
done
