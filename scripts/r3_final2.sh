# round 3, last evidence pass on the final tree: GPU suite, driver-shaped bench, decode windows of the headline,
# GPT-2-XL and the TP=8 shard (batch 512)
mkdir -p gpurun_out/final2
T="--timeout 300 --timeout-method thread"
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/final2/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/final2/bench.log 2>&1 || exit $?
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/final2/llama7b_tp1_window.summary.txt
BENCH_ARGS="--model gpt2-xl --steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/final2/gpt2xl_window.summary.txt
BENCH_ARGS="--simulate-tp 8 --steps 1 --warmup 1 --secondary none" ANCHOR=sample_cand SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/final2/tp8sim_window.summary.txt
rm -f gpurun_out/tp1_window.csv
tail -n 2 gpurun_out/final2/pytest_gpu.log; tail -n 1 gpurun_out/final2/bench.log | cut -c1-300
