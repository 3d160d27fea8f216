set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/kernels2.log 2>&1; tail -3 gpurun_out/kernels2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 && echo SMOKE_OK &&
for C in 1 64 256; do timeout -k 10 600 python bench.py --mode engine --steps 2 --warmup 1 --concurrency $C > gpurun_out/bench2_c$C.log 2>&1 || exit 1; tail -1 gpurun_out/bench2_c$C.log; done
