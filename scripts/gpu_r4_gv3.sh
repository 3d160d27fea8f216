#!/bin/bash
# dp4 GEMV variants per Llama-3-8B decode shape at M=2
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
GEMV_M=2 GEMV_VARIANTS=1,3,5,9 timeout -k 10 500 python -u scripts/gemv_variants.py > gpurun_out/gv_var2.log 2>&1 && grep "M=2" gpurun_out/gv_var2.log
