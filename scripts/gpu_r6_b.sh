set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/bs_bench.py --abl --m 8192 256 > gpurun_out/r6b_abl.log 2>&1; cat gpurun_out/r6b_abl.log
bash scripts/gpu_pmc_run.sh scripts/pmc_bs.py gpurun_out/r6b_pmc
