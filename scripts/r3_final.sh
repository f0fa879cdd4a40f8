# round 3 end-of-session evidence: the whole GPU suite, the driver-shaped bench, a rocprofv3 --stats run of the
# bench and steady-state decode windows (Llama-2-7B TP=1, GPT-2-XL, fp8 70B TP=8 shard)
mkdir -p gpurun_out/final
T="--timeout 300 --timeout-method thread"
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/final/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/final/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/final/prof.log 2>&1 || exit $?
rm -f gpurun_out/final/prof/*kernel_trace.csv
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/final/llama7b_tp1_window.summary.txt
BENCH_ARGS="--model gpt2-xl --steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/final/gpt2xl_window.summary.txt
tail -n 3 gpurun_out/final/pytest_gpu.log; tail -n 1 gpurun_out/final/bench.log | cut -c1-400
