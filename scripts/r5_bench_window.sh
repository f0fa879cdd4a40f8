# round 5: headline bench on the current tree, then the steady-state decode window of Llama-2-7B TP=1
set -u
mkdir -p gpurun_out/r5b
timeout -k 10 420 python bench.py --steps 5 --warmup 2 > gpurun_out/r5b/bench.log 2>&1 || { tail -30 gpurun_out/r5b/bench.log; exit 1; }
tail -1 gpurun_out/r5b/bench.log
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r5b/llama7b_tp1_window.summary.txt
cp gpurun_out/tp1_window.csv gpurun_out/r5b/llama7b_tp1_window.csv
rm -f gpurun_out/tp1_window.csv
cat gpurun_out/r5b/llama7b_tp1_window.summary.txt
