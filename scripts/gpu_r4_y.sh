#!/bin/bash
# Mixtral-8x7B function calling C=32 (BASELINE config 4): throughput + rocprof kernel summary
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -c "
import os; from localai_amd.models import synth
p = os.path.join(os.environ['LOCALAI_AMD_CACHE'], 'mixtral-8x7b.gguf'); os.makedirs(os.path.dirname(p), exist_ok=True)
synth.write_model(p, 'mixtral-8x7b') if not os.path.exists(p) else None; print('model ok')" > gpurun_out/y_gen.log 2>&1 &&
timeout -k 10 500 python -u scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32 --max-tokens 128 > gpurun_out/y_fc.log 2>&1 && tail -1 gpurun_out/y_fc.log | cut -c1-400 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/la_prof/fc -o run --output-format csv -- python3 $R/scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32 --max-tokens 128 --waves 1 --checks 2 > $R/gpurun_out/y_prof.log 2>&1 &&
python3 $R/scripts/prof_summary.py /tmp/la_prof/fc "Mixtral-8x7B function calling, C=32, GBNF-constrained (round 4)" > $R/gpurun_out/y_prof_fc.md && head -30 $R/gpurun_out/y_prof_fc.md
