set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=4
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --stats -d /tmp/pmc$i -o run --output-format csv -- python3 $R/scripts/pmc_kernels.py > $R/gpurun_out/pmc$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $R/gpurun_out/pmc$i.log; continue; }
  mkdir -p $R/gpurun_out/pmc$i && cp $(find /tmp/pmc$i -name "*counter_collection.csv" | head -1) $R/gpurun_out/pmc$i/ 2>/dev/null
  echo "pass $i ok"
done
