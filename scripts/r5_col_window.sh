# steady-state decode window of the simulated TP=8 shard with the column-chunked schedule
set -u
mkdir -p gpurun_out/r5c
export LLMSS_TP_COL=${COL:-4}
BENCH_ARGS="--simulate-tp 8 --sim-comm 15,150 --steps 1 --warmup 1 --secondary none" ANCHOR=sample_cand SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r5c/col${COL:-4}_window.summary.txt
cp gpurun_out/tp1_window.csv gpurun_out/r5c/col${COL:-4}_window.csv
rm -f gpurun_out/tp1_window.csv
head -30 gpurun_out/r5c/col${COL:-4}_window.summary.txt
