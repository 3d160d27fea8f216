export PYTHONUNBUFFERED=1
BENCH_DUMP_GEMM=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r6e_bs.log 2> gpurun_out/r6e_bs.err || { tail -20 gpurun_out/r6e_bs.err; exit 1; }
tail -1 gpurun_out/r6e_bs.log; grep "choice" gpurun_out/r6e_bs.err | head -40
LOCALAI_AMD_BS=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r6e_nobs.log 2> gpurun_out/r6e_nobs.err; tail -1 gpurun_out/r6e_nobs.log
