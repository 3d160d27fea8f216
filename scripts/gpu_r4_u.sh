#!/bin/bash
# Mixtral C=32: 4- vs 8-wave MoE workgroups for 17..32-row batches (A/B); MoE tests both ways
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-330; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step u_kern.log 300 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "moe or mixtral"
LOCALAI_AMD_MOE_TUNE=0,11 step u_kern11.log 300 $PT tests/test_kernels_gpu.py -k "moe_grouped"
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/u_gen.log 2>&1 &&
for cfg in "0,8" "0,11" "0,8" "0,11"; do
  LOCALAI_AMD_MOE_TUNE=$cfg step u_mx32_${cfg/,/_}.log 400 python -u bench.py --mode engine --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 32 --max-tokens 128
done
