# round 3: steady-state decode windows (compact kernel traces) for the fp8 70B TP=8 shard and GPT-2-XL
set -e
mkdir -p gpurun_out/windows
for cfg in "fp8_70b_tp8sim|sample_cand|--model llama2-70b --fp8 --simulate-tp 8 --steps 1 --warmup 1 --secondary none" \
           "gpt2xl|sample_v3|--model gpt2-xl --steps 2 --warmup 1 --secondary none"; do
  name=${cfg%%|*}; rest=${cfg#*|}; anchor=${rest%%|*}; args=${rest#*|}
  BENCH_ARGS="$args" ANCHOR=$anchor SKIP=0.6 SPAN=30000 bash scripts/tp1_trace.sh
  cp gpurun_out/tp1_window.csv gpurun_out/windows/$name.csv
  python scripts/step_breakdown.py gpurun_out/windows/$name.csv > gpurun_out/windows/$name.summary.txt
  tail -1 gpurun_out/tp1_tr.log | cut -c1-300
done
