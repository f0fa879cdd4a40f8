# round 5: is the priority comm stream what slows the overlapped decode schedules under the spin-kernel comm model?
set -u
mkdir -p gpurun_out/r5p
for cfg in "4 -1" "4 0" "0 0"; do
  set -- $cfg
  LLMSS_TP_COL=$1 LLMSS_COMM_PRIO=$2 timeout -k 10 400 python bench.py --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 \
    --secondary none > gpurun_out/r5p/col$1_prio$2.log 2>&1 || { tail -20 gpurun_out/r5p/col$1_prio$2.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5p/col$1_prio$2.log').read().strip().splitlines()[-1]); print('COL=$1 PRIO=$2', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
