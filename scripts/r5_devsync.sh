# round 5 (historical: csrc/sync.hip and LLMSS_TP_DEVSYNC were removed again, profiles/r5_tbo): device-flag stream hand-off - probe, GPU tests of the overlapped schedules, TP=8 sim
set -u
mkdir -p gpurun_out/r5d
T="--timeout 300 --timeout-method thread"
timeout -k 10 60 python bench/xq_probe.py --us 20 --side-us 10 --arms serial,tbo,tbo_devsync > gpurun_out/r5d/probe.json 2>&1 || { tail -20 gpurun_out/r5d/probe.json; exit 1; }
cat gpurun_out/r5d/probe.json
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py -q -x -rf $T > gpurun_out/r5d/comm_tests.log 2>&1 || { tail -30 gpurun_out/r5d/comm_tests.log; exit 1; }
tail -1 gpurun_out/r5d/comm_tests.log
for cfg in "tbo_devsync 1" "tbo_events 0"; do
  set -- $cfg
  LLMSS_TP_COL=0 LLMSS_TP_DECODE_OVERLAP_MIN=128 LLMSS_TP_DEVSYNC=$2 timeout -k 10 400 python bench.py --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 --secondary none > gpurun_out/r5d/$1.log 2>&1 || { tail -20 gpurun_out/r5d/$1.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5d/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
