# round 6: Llama-2-70B fp8 TP=8 shard decode window (timed steps: the last ~8 % of the trace) with the MX hand-off
set -u
mkdir -p gpurun_out/r6mx
BENCH_ARGS="--model llama2-70b --fp8 --simulate-tp 8 --secondary none --steps 1 --warmup 1" ANCHOR=sample_cand SKIP=0.6 SPAN=20000 bash scripts/tp1_trace.sh || exit $?
python3 scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r6mx/llama70b_fp8_tp8sim_window.summary.txt
rm -f gpurun_out/tp1_window.csv
head -16 gpurun_out/r6mx/llama70b_fp8_tp8sim_window.summary.txt
