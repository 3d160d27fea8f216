# prefill chunk size A/B on the default HTTP bench (prefix-unique waves)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
for cfg in "--batch-tokens 8192" "--batch-tokens 16384" "--batch-tokens 4096" "--batch-tokens 8192"; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 $cfg > gpurun_out/b_sched.log 2>&1 || exit 1
  echo "$cfg :: $(tail -1 gpurun_out/b_sched.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ttft_ms"], d["p90_ttft_ms"])')"
done
