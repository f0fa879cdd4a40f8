# round 5: the TP=8 shard (batch 512, rank-0 compute) with a modelled all-reduce (15 us + bytes / 150 GB/s on the
# issuing stream): one all-reduce per row-parallel output vs the column-chunked schedule (LLMSS_TP_COL=C)
set -u
mkdir -p gpurun_out/r5t
for cfg in ${CFGS:-0 4 2 8}; do
  LLMSS_TP_COL=$cfg timeout -k 10 400 python bench.py --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 \
    --secondary none > gpurun_out/r5t/col$cfg.log 2>&1 || { tail -20 gpurun_out/r5t/col$cfg.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5t/col$cfg.log').read().strip().splitlines()[-1]); print('LLMSS_TP_COL=$cfg', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
