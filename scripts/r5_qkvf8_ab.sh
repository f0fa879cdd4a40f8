# round 5: A/B of the fp8 QKV RoPE / KV-write epilogue on the 70B fp8 TP=8 shard (LLMSS_QKV_EPI=0 vs 1, twice each)
set -u
mkdir -p gpurun_out/r5q8
for i in 1 2; do
  for e in 0 1; do
    LLMSS_QKV_EPI=$e timeout -k 10 400 python bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/r5q8/ab_epi${e}_$i.log 2>&1 || { tail -20 gpurun_out/r5q8/ab_epi${e}_$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5q8/ab_epi${e}_$i.log').read().strip().splitlines()[-1]); print('epi=$e run $i', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
  done
done
