# round 6: steady-state decode windows (rocprofv3 kernel trace, 12 ms after 60 % of the run) of GPT-2-XL and
# Llama-2-7B TP=1 on the current tree; per-kernel time per window (scripts/step_breakdown.py)
set -u
mkdir -p gpurun_out/r6w
for m in gpt2-xl llama2-7b; do
  BENCH_ARGS="--model $m --secondary none --steps 2 --warmup 1" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
  python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r6w/${m}_window.summary.txt
  rm -f gpurun_out/tp1_window.csv
  cat gpurun_out/r6w/${m}_window.summary.txt | head -14
done
