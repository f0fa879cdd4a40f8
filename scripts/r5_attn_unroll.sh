# round 5 (historical: LLMSS_ATTN_UNROLL was a temporary hook, removed after this A/B): decode-attention pipeline depth in the decode step
set -u
mkdir -p gpurun_out/r5au
for u in 11 12 2; do
  LLMSS_ATTN_UNROLL=$u timeout -k 10 600 python bench.py --steps 4 --warmup 1 > gpurun_out/r5au/u$u.log 2>&1 || { tail -20 gpurun_out/r5au/u$u.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5au/u$u.log').read().strip().splitlines()[-1]); s=d['secondary']; print('u$u', d['value'], d['p50_tpot_ms'], s['engine_direct']['value'], s['engine_direct']['p50_tpot_ms'])"
done
