#!/bin/bash
# Counter passes over a launch driver (kernel-trace/stats only; each pass its own run):
#   bash scripts/gpu_pmc_run.sh scripts/pmc_bs.py gpurun_out/bspmc
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && DRV=$1 && OUT=$R/$2 && mkdir -p $OUT
timeout -k 10 120 python3 $DRV > $OUT/drv.log 2>&1 || { tail -5 $OUT/drv.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/pmcrun$i -o run --output-format csv -- python3 $R/$DRV > $OUT/pass$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $OUT/pass$i.log; continue; }
  cp $(find /tmp/pmcrun$i -name "*counter_collection.csv" | head -1) $OUT/counters$i.csv 2>/dev/null
  cp $(find /tmp/pmcrun$i -name "*kernel_stats.csv" | head -1) $OUT/stats$i.csv 2>/dev/null
  echo "pass $i ok"
done
