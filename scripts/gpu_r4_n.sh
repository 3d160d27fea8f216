#!/bin/bash
# MoE wide tile default (64 rows x 8 waves): tests, Mixtral HTTP C=256, decode profile
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step n_kern.log 300 $PT tests/test_kernels_gpu.py -k "moe"
step n_eng.log 400 $PT tests/test_engine_gpu.py -k "mixtral"
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/n_gen.log 2>&1 &&
step n_mx256.log 700 python -u bench.py --mode http --preset mixtral-8x7b --steps 2 --warmup 1 --concurrency 256 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/mx -o run --output-format csv -- python3 $R/bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 0 --concurrency 256 --max-tokens 64 > $R/gpurun_out/n_prof.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/mx "Engine C=256, Mixtral-8x7B Q4_K_M (round 4, 64-row x 8-wave MoE tiles)" --steady 32 --by-grid 32 > $R/gpurun_out/n_prof_mx256.md && grep -A14 "Decode steady" $R/gpurun_out/n_prof_mx256.md
