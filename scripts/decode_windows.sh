# steady-state decode windows (compact kernel traces) for the headline config and the TP=8 shard
set -e
mkdir -p gpurun_out/windows
for cfg in "tp1|--secondary none" "tp8sim|--simulate-tp 8" "gpt2xl|--model gpt2-xl --secondary none"; do
  name=${cfg%%|*}; args=${cfg#*|}
  BENCH_ARGS="$args" ANCHOR=sample_v3 SKIP=0.7 SPAN=11000 bash scripts/tp1_trace.sh
  cp gpurun_out/tp1_window.csv gpurun_out/windows/$name.csv
  tail -1 gpurun_out/tp1_tr.log | cut -c1-200
done
