set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or sample" > gpurun_out/pytest_attn.log 2>&1 && tail -1 gpurun_out/pytest_attn.log &&
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1 && cat gpurun_out/attn_bench.log &&
cp localai_amd/ops/_la_kernels.so /tmp/new.so && cp build_old/_la_kernels.so localai_amd/ops/_la_kernels.so && echo OLD: &&
timeout -k 10 300 python -u scripts/attn_bench.py; rc=$?; cp /tmp/new.so localai_amd/ops/_la_kernels.so; exit $rc
