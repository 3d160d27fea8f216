#!/bin/bash
# Round-5 prefill GEMM diagnosis: stamps, then variant timings one process per group, stopping at
# the first failure (each step bounded).
set -e
cd "$(dirname "$0")/.."
O=gpurun_out
timeout -k 10 120 python -u scripts/pp_abl.py --stamp --shapes gate_up --m 8192 > $O/pp_stamp.log 2>&1
timeout -k 10 200 python -u scripts/pp_abl.py --only base,slp,gm1,gm4 --m 8192 2048 --bf16 > $O/pp_var.log 2>&1
for v in abl1 abl2 abl4 abl8 abl16 abl10 abl30; do
  echo "== $v" >> $O/pp_abl3.log
  timeout -k 10 120 python -u scripts/pp_abl.py --only base,$v --m 8192 --rounds 3 >> $O/pp_abl3.log 2>&1
done
