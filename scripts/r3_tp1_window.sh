# round 3: steady-state decode window of the headline config (Llama-2-7B TP=1, batch 64) and the startup cost of
# the TP=8 shard engine (autotune + graph capture at 25 buckets), wall-clocked
set -e
mkdir -p gpurun_out/windows
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh
cp gpurun_out/tp1_window.csv gpurun_out/windows/tp1.csv
python scripts/step_breakdown.py gpurun_out/windows/tp1.csv > gpurun_out/windows/tp1.summary.txt
t0=$(date +%s.%N)
timeout -k 10 600 python bench.py --simulate-tp 8 --steps 1 --warmup 0 --secondary none > gpurun_out/tp8sim_startup.log 2>&1
t1=$(date +%s.%N)
echo "tp8sim total wall s: $(echo "$t1 - $t0" | bc)" >> gpurun_out/tp8sim_startup.log
