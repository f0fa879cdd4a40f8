# round 5: two-micro-batch decode with micro-batch B on a second compute stream (LLMSS_TBO_STREAMS=2) vs one stream,
# TP=8 shard under the comm model; then the GPU tests of the overlapped schedules
set -u
mkdir -p gpurun_out/r5t2
T="--timeout 300 --timeout-method thread"
for cfg in tbo1:1 tbo2:2; do
  set -- ${cfg/:/ }
  LLMSS_TP_COL=0 LLMSS_TP_DECODE_OVERLAP_MIN=128 LLMSS_TBO_STREAMS=$2 timeout -k 10 400 python bench.py --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 --secondary none > gpurun_out/r5t2/$1.log 2>&1 || { tail -20 gpurun_out/r5t2/$1.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5t2/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
LLMSS_TBO_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py -q -x -rf $T > gpurun_out/r5t2/comm_tests.log 2>&1 || { tail -30 gpurun_out/r5t2/comm_tests.log; exit 1; }
tail -1 gpurun_out/r5t2/comm_tests.log
