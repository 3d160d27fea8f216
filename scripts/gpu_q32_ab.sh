#!/bin/bash
# q32 GEMM numerics + engine-mode C=256 A/B (q32 candidates on / off) on one box
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gemm_tile_gpu.py -x -q --timeout 300 > gpurun_out/t_gemm.log 2>&1 || { tail -30 gpurun_out/t_gemm.log; exit 1; }
tail -3 gpurun_out/t_gemm.log
BENCH_DUMP_GEMM=1 timeout -k 10 600 python -u bench.py --mode engine --steps 4 --warmup 2 > gpurun_out/b_eng_q32.log 2>&1 || { tail -20 gpurun_out/b_eng_q32.log; exit 1; }
tail -1 gpurun_out/b_eng_q32.log
LOCALAI_AMD_Q32=0 timeout -k 10 600 python -u bench.py --mode engine --steps 4 --warmup 2 > gpurun_out/b_eng_noq32.log 2>&1 || { tail -20 gpurun_out/b_eng_noq32.log; exit 1; }
tail -1 gpurun_out/b_eng_noq32.log
