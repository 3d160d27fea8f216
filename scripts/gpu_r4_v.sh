#!/bin/bash
# Mixtral HTTP C=256: prefill GEMMs (dense per-expert path included) on the library vs the tile kernel
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -1 gpurun_out/$log | cut -c1-420; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/v_gen.log 2>&1 &&
for g in blas tile blas tile; do
  LOCALAI_AMD_PREFILL_GEMM=$g step v_mx_$g.log 500 python -u bench.py --mode http --preset mixtral-8x7b --steps 1 --warmup 1 --concurrency 256 --max-tokens 64
done
