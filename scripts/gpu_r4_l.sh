#!/bin/bash
# re-run of the round-end rehearsal failures: deterministic GroupNorm stats, AR world 8, fused-norm tests
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() { local log=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$log 2>&1; local rc=$?; tail -2 gpurun_out/$log | cut -c1-600; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$log | head -20; tail -30 gpurun_out/$log; exit $rc; }; }
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step l_sd.log 600 $PT tests/test_sd.py tests/test_sdxl.py -m gpu
step l_kern.log 300 $PT tests/test_kernels_gpu.py -k "fused_norm"
step l_ar.log 600 $PT tests/test_custom_allreduce.py
step l_det.log 300 python -u scripts/determinism_probe.py --deterministic
