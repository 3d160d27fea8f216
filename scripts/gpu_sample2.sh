# sampler passes: sampling kernel tests, engine sampling tests, sampler timing probe
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "sample or mirostat or penalt or grammar or seed" > gpurun_out/pytest_sample.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_sample.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/sample_bench.py > gpurun_out/sample_bench.log 2>&1 && cat gpurun_out/sample_bench.log
