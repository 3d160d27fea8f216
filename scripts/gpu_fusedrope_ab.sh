# A/B: RoPE+KV-append fused into decode attention vs separate rope_kv launch (engine C=1, C=64, C=256)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export LOCALAI_AMD_CACHE=/tmp/la_cache
for c in 1 64 256; do
  for f in 0 1; do
    LOCALAI_AMD_FUSED_ROPE=$f timeout -k 10 300 python bench.py --mode engine --steps 2 --warmup 1 --concurrency $c --max-tokens 128 > gpurun_out/ab_rope_c${c}_f${f}.log 2>&1 || exit $?
    echo "C=$c fused=$f $(tail -1 gpurun_out/ab_rope_c${c}_f${f}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
