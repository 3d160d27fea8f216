#!/bin/bash
# MIOpen determinism, setprio A/B, mixed grammar batch with expanded riders, Q5_K_M test
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }



step t_q5.log 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "non_tile or rides"
step b_eng.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
LOCALAI_AMD_KLIB=_la_kernels_prio.so step b_eng_prio.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
step b_eng2.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
LOCALAI_AMD_KLIB=_la_kernels_prio.so step b_eng_prio2.log 400 python -u bench.py --mode engine --steps 4 --warmup 2
step mixed_b.log 600 python -u scripts/mixed_batch_bench.py
LOCALAI_AMD_TRACE=gpurun_out/trace_http.json step b_http_tr.log 400 python -u bench.py --steps 2 --warmup 1
LOCALAI_AMD_TRACE=gpurun_out/trace_eng.json step b_eng_tr.log 400 python -u bench.py --mode engine --steps 2 --warmup 1
