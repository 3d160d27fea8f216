# engine-mode concurrency sweep on HEAD (Llama-3-8B Q4_K_M random-init): C = 1, 2, 16, 64
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
for c in 1 2 16 64; do
  timeout -k 10 400 python -u bench.py --mode engine --steps 2 --warmup 1 --concurrency $c --max-tokens 128 > gpurun_out/s3_conc_$c.log 2>&1 || exit $?
  echo "C=$c $(tail -1 gpurun_out/s3_conc_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "tok/s p50", d.get("p50_ttft_ms"), "ms")')"
done
