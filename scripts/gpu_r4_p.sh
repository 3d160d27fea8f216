#!/bin/bash
# dense per-expert MoE prefill + anyres gather: tests, Mixtral HTTP C=256 A/B
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-400; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step p_kern.log 300 $PT tests/test_kernels_gpu.py -k "gather or moe or clip"
step p_eng.log 500 $PT tests/test_engine_gpu.py -k "mixtral or llava"
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/p_gen.log 2>&1 &&
step p_mx256.log 700 python -u bench.py --mode http --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256 &&
LOCALAI_AMD_MOE_DENSE_MIN_T=1000000 step p_mx256_grouped.log 700 python -u bench.py --mode http --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256
