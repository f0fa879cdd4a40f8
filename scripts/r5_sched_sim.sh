# round 5: the overlapped decode schedules under the TP=8 comm model with the comm stream at normal priority
# (each line: env assignments for one run)
set -u
mkdir -p gpurun_out/r5s
while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 400 python bench.py --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 \
    --secondary none > gpurun_out/r5s/$name.log 2>&1 || { tail -20 gpurun_out/r5s/$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5s/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done <<'LIST'
col2 LLMSS_TP_COL=2
tbo LLMSS_TP_COL=0 LLMSS_TP_DECODE_OVERLAP_MIN=128
rsag LLMSS_TP_COL=0 LLMSS_TP_RSAG=1
tbo_prio1 LLMSS_TP_COL=0 LLMSS_TP_DECODE_OVERLAP_MIN=128 LLMSS_COMM_PRIO=-1
LIST
