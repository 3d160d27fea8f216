#!/bin/bash
# determinism probe (SDXL toy), small-batch attention split A/B, mixed grammar batch test +
# bench, weight-nt A/B, Mixtral FC
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
step det_xl.log 300 python -u scripts/determinism_probe.py --size tiny-xl
step det_sd.log 300 python -u scripts/determinism_probe.py --size tiny
LOCALAI_AMD_DEC_SPLIT_SHORT=16 step t_attn_split.log 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attn_decode
step attn_ns.log 200 python -u scripts/attn_bench.py
LOCALAI_AMD_DEC_SPLIT_SHORT=16 step attn_s.log 200 python -u scripts/attn_bench.py
grep -h "B=  1\|B=  2" gpurun_out/attn_ns.log gpurun_out/attn_s.log
step t_mixed.log 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "rides"
step b_eng.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
LOCALAI_AMD_KLIB=_la_kernels_wnt.so step b_eng_wnt.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
step b_eng2.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
step fc_mx.log 800 python -u scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32 --max-tokens 128
