# the other BASELINE configs on the round-5 tree (one MI355X), then the 70B fp8 TP=8 shard's decode window
set -u
mkdir -p gpurun_out/r5c2
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" --secondary none > gpurun_out/r5c2/$n.log 2>&1 || { tail -20 gpurun_out/r5c2/$n.log; exit 1; }; echo "$n $(grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' gpurun_out/r5c2/$n.log | tr '\n' ' ')"; }
run llama7b_tp8sim --simulate-tp 8 --steps 2 --warmup 1 &&
LLMSS_TP_DECODE_OVERLAP_MIN=128 run llama7b_tp8sim_comm_tbo --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 &&
run llama13b_tp1 --model llama2-13b --steps 2 --warmup 1 &&
run llama13b_tp8sim --model llama2-13b --simulate-tp 8 --steps 2 --warmup 1 &&
LLMSS_TP_DECODE_OVERLAP_MIN=128 run llama13b_tp8sim_comm_tbo --model llama2-13b --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1 &&
run llama70b_fp8_tp8sim --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r5c2/tr70 -o run --output-format csv -- python3 bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 1 --warmup 1 --secondary none > gpurun_out/r5c2/tr70.log 2>&1 || { tail -20 gpurun_out/r5c2/tr70.log; exit 1; }
python scripts/trace_window.py gpurun_out/r5c2/tr70/run_kernel_trace.csv gpurun_out/r5c2/llama70b_fp8_tp8sim_window.csv --skip-frac 0.6 --anchor sample_cand --span-us 20000
rm -f gpurun_out/r5c2/tr70/*kernel_trace.csv
python scripts/step_breakdown.py gpurun_out/r5c2/llama70b_fp8_tp8sim_window.csv > gpurun_out/r5c2/llama70b_fp8_tp8sim_window.summary.txt
head -25 gpurun_out/r5c2/llama70b_fp8_tp8sim_window.summary.txt
