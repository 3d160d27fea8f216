#!/bin/bash
# TP rehearsals (ranks sharing the one GPU) with decode graphs + per-row logits vs TP=1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r5_tp.log 2>&1
