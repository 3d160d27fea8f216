#!/bin/bash
# Round-end rehearsal (GPU suite, smoke, benches, HTTP profile) followed by the SD-1.5 bench
set -o pipefail
bash scripts/gpu_round_r2c.sh && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 python -u scripts/sd_bench.py --steps 20 --runs 3 > gpurun_out/sd_bench.log 2>&1 && tail -1 gpurun_out/sd_bench.log
