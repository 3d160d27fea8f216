# PMC counters for the skinny GEMM (counter runs use --kernel-trace/--stats only, no other traces).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc VALUBusy MemUnitBusy --kernel-trace --stats -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/scripts/skinny_only.py > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE VALUUtilization --kernel-trace --stats -d $R/gpurun_out/pmc2 -o run --output-format csv -- python3 $R/scripts/skinny_only.py > $R/gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES --kernel-trace --stats -d $R/gpurun_out/pmc3 -o run --output-format csv -- python3 $R/scripts/skinny_only.py > $R/gpurun_out/pmc3.log 2>&1 || exit 1
ls -R $R/gpurun_out/pmc1 | head
