mkdir -p gpurun_out
export LLMSS_AUTOTUNE=0
run() { name=$1; shift; timeout -k 10 200 "$@" > gpurun_out/diag_$name.log 2>&1 || { echo "$name failed"; exit 1; }; echo "$name $(tail -1 gpurun_out/diag_$name.log | grep -o '"p50_tpot_ms": [0-9.]*')"; }
LLMSS_SIM_COMM_OP=touch run graph_tbo_touch python bench.py --simulate-tp 8 --sim-comm 0.1,100000 --steps 1 --warmup 0
run eager_tbo_sleep python bench.py --simulate-tp 8 --sim-comm 0.1,100000 --steps 1 --warmup 0 --no-graphs
LLMSS_TP_DECODE_OVERLAP_MIN=0 run eager_off_sleep python bench.py --simulate-tp 8 --sim-comm 0.1,100000 --steps 1 --warmup 0 --no-graphs
LLMSS_SIM_COMM_OP=touch LLMSS_TP_DECODE_OVERLAP_MIN=0 run graph_off_touch python bench.py --simulate-tp 8 --sim-comm 0.1,100000 --steps 1 --warmup 0
