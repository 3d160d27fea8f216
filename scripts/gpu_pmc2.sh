# counter passes (kernel-trace/stats only; each pass its own run) over scripts/pmc_kernels.py
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/pmc_kernels.py > gpurun_out/pmck.log 2>&1 || { tail -5 gpurun_out/pmck.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "FETCH_SIZE WRITE_SIZE" "VALUBusy MemUnitBusy" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/pmc$i -o run --output-format csv -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $R/gpurun_out/pmc$i.log; continue; }
  mkdir -p $R/gpurun_out/pmc$i && cp $(find /tmp/pmc$i -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc$i/ 2>/dev/null
  cp $(find /tmp/pmc$i -name "*kernel_stats.csv" | head -1) $R/gpurun_out/pmc$i/ 2>/dev/null
  echo "pass $i ok"
done
ls $R/gpurun_out/pmc*/
