#!/bin/bash
# counter passes (kernel-trace + stats only, one pass per run) over scripts/pmc_moe.py
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out/pmcm
timeout -k 10 300 python3 scripts/pmc_moe.py > gpurun_out/pmcm/drv.log 2>&1 || { tail -5 gpurun_out/pmcm/drv.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/pmcm_$i -o run --output-format csv -- python3 $R/scripts/pmc_moe.py > $R/gpurun_out/pmcm/pass$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $R/gpurun_out/pmcm/pass$i.log; continue; }
  cp $(find /tmp/pmcm_$i -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmcm/counters$i.csv 2>/dev/null
  cp $(find /tmp/pmcm_$i -name "*kernel_stats.csv" | head -1) $R/gpurun_out/pmcm/stats$i.csv 2>/dev/null
  echo "pass $i ok"
done
