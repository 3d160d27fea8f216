#!/bin/bash
# Mixtral-8x7B engine C=256 decode profile (where do ~37 ms per step go?)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/k_gen.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/mx -o run --output-format csv -- python3 $R/bench.py --mode engine --preset mixtral-8x7b --steps 1 --warmup 0 --concurrency 256 --max-tokens 64 > $R/gpurun_out/k_prof.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/mx "Engine C=256, Mixtral-8x7B Q4_K_M (round 4)" --steady 32 --by-grid 32 > $R/gpurun_out/k_prof_mx256.md && tail -60 $R/gpurun_out/k_prof_mx256.md
