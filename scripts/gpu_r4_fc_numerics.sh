#!/bin/bash
# function-calling validity on the GPU (tiny SPM MoE, Mixtral-8x7B, Llama-3-8B) + the tightened
# numerics tests (headline oracle with logit bounds, SD-family vs fp32) + smoke
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -3 gpurun_out/$log | cut -c1-900; [ $rc -eq 0 ] || { tail -30 gpurun_out/$log; exit $rc; }; }
step t_num.log 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "oracle" tests/test_sd.py tests/test_sdxl.py tests/test_flux.py tests/test_sd3.py
grep -h "numerics\|denoiser vs" gpurun_out/t_num.log
step smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step fc_tiny.log 300 python -u scripts/fc_bench.py --preset tiny-mixtral-spm --concurrency 8 --waves 1
step fc_mx.log 800 python -u scripts/fc_bench.py --preset mixtral-8x7b --concurrency 32
grep INVALID gpurun_out/fc_mx.log | head -3 | cut -c1-700
step fc_8b.log 500 python -u scripts/fc_bench.py --preset llama3-8b --concurrency 32
