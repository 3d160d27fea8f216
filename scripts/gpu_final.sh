# Round-end rehearsal on HEAD: GPU tests (one process), smoke(), default bench line, DP=2 launch
# rehearsal (2 ranks share the one GPU over gloo), and a C=256 HTTP-path kernel profile summary.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log | cut -c1-330 &&
BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 64 --max-tokens 64 > gpurun_out/b_dp2.log 2>&1 && tail -1 gpurun_out/b_dp2.log | cut -c1-250 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/h256 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --concurrency 256 --max-tokens 128 > $R/gpurun_out/prof_h256.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/h256 "HTTP C=256, Llama-3-8B Q4_K_M" > $R/gpurun_out/prof_h256.md && echo PROF_OK
