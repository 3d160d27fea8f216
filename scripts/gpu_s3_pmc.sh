#!/bin/bash
# counter passes (kernel-trace + stats only, one pass per run) over scripts/pmc_r3_hot.py
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/pmc3
timeout -k 10 120 python3 scripts/pmc_r3_hot.py > gpurun_out/pmc3/drv.log 2>&1 || { tail -5 gpurun_out/pmc3/drv.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/pmc3_$i -o run --output-format csv -- python3 $R/scripts/pmc_r3_hot.py > $R/gpurun_out/pmc3/pass$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $R/gpurun_out/pmc3/pass$i.log; continue; }
  cp $(find /tmp/pmc3_$i -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc3/counters$i.csv 2>/dev/null
  cp $(find /tmp/pmc3_$i -name "*kernel_stats.csv" | head -1) $R/gpurun_out/pmc3/stats$i.csv 2>/dev/null
  echo "pass $i ok"
done
