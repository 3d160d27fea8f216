# PMC counters for the mid-M GEMM (counter runs: --pmc + --kernel-trace/--stats only).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-trace --stats -d $R/gpurun_out/pmcm1 -o run --output-format csv -- python3 $R/scripts/mid_only.py > $R/gpurun_out/pmcm1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --stats -d $R/gpurun_out/pmcm2 -o run --output-format csv -- python3 $R/scripts/mid_only.py > $R/gpurun_out/pmcm2.log 2>&1 || exit 1
echo PMC_OK
