set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python bench.py --mode engine --preset llama3-8b-q8_0 --steps 2 --warmup 1 --concurrency 1 --max-tokens 256 > gpurun_out/b_q8_c1.log 2>&1 && tail -1 gpurun_out/b_q8_c1.log | cut -c1-150 &&
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "wide or multistep or families" > gpurun_out/pytest_wide.log 2>&1; rc=$?; grep -E "FAIL|passed|failed" gpurun_out/pytest_wide.log | tail -4; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python bench.py > gpurun_out/b_wide.log 2>&1 && tail -1 gpurun_out/b_wide.log | cut -c1-330
timeout -k 10 600 python bench.py --decode-steps 8 > gpurun_out/b_k8.log 2>&1 && tail -1 gpurun_out/b_k8.log | cut -c1-330
done
