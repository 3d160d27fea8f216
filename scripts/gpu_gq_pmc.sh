#!/bin/bash
# counter passes over scripts/gq_pmc.py (kernel-trace/stats only; each pass its own run)
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/gqpmc
timeout -k 10 120 python3 scripts/gq_pmc.py > gpurun_out/gqpmc/drv.log 2>&1 || { tail -5 gpurun_out/gqpmc/drv.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/gqpmc$i -o run --output-format csv -- python3 $R/scripts/gq_pmc.py > $R/gpurun_out/gqpmc/pass$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $R/gpurun_out/gqpmc/pass$i.log; continue; }
  cp $(find /tmp/gqpmc$i -name "*counter_collection.csv" | head -1) $R/gpurun_out/gqpmc/counters$i.csv 2>/dev/null
  cp $(find /tmp/gqpmc$i -name "*kernel_stats.csv" | head -1) $R/gpurun_out/gqpmc/stats$i.csv 2>/dev/null
  echo "pass $i ok"
done
