#!/bin/bash
# two-shot all-reduce: exactness (two ranks sharing the GPU), latency, TP engine rehearsal
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce.py tests/test_tp_gpu.py "tests/test_kernels_gpu.py::test_clip_image_preprocess_kernel_matches_pil" tests/test_engine_gpu.py::test_llava_on_gpu -m gpu -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_ar2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s2_ar2.log | tail -6
[ $rc -eq 0 ] || exit $rc
LOCALAI_AMD_AR_SAME_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 scripts/ar_check.py > gpurun_out/s2_ar2_check.log 2>&1
rc=$?
grep AR_OK gpurun_out/s2_ar2_check.log
[ $rc -eq 0 ] || exit $rc
export LOCALAI_AMD_CACHE=/tmp/la_cache
timeout -k 10 600 python -u scripts/mixed_batch_bench.py > gpurun_out/s2_mixed.log 2>&1
rc=$?
grep "decode" gpurun_out/s2_mixed.log
[ $rc -eq 0 ] || exit $rc
# headline A/B on one box: the round-3 tile GEMM path vs the round-2 path (hipBLASLt on bf16 copies)
timeout -k 10 400 python3 bench.py --steps 8 --warmup 2 > gpurun_out/s2_bench_tile.log 2>&1 && tail -1 gpurun_out/s2_bench_tile.log | cut -c1-330 &&
LOCALAI_AMD_TILE_GEMM=0 timeout -k 10 400 python3 bench.py --steps 8 --warmup 2 > gpurun_out/s2_bench_r2path.log 2>&1 && tail -1 gpurun_out/s2_bench_r2path.log | cut -c1-330
