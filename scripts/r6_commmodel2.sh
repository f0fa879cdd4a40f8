# round 6: the row-sharded (reduce-scatter / all-gather) and column-chunked decode schedules under both comm models
set -u
mkdir -p gpurun_out/r6cm
run() {
  timeout -k 10 500 python3 bench.py --simulate-tp 8 --secondary none --steps 2 --warmup 1 "$@" > gpurun_out/r6cm/$name.json 2> gpurun_out/r6cm/$name.err \
    || { tail -20 gpurun_out/r6cm/$name.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6cm/$name.json')); print('$name', d['value'], d['p50_tpot_ms'], d['config']['parallelism'])"
}
export LLMSS_TP_RSAG=1
name=spin_rsag run --sim-comm 15,150 && name=ch32_rsag run --sim-comm 15,150,32
export LLMSS_TP_RSAG=auto LLMSS_TP_COL=4
name=spin_col4 run --sim-comm 15,150 && name=ch32_col4 run --sim-comm 15,150,32
