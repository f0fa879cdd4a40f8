# streamed gRPC (GenerateStream, open loop) and closed-loop unary serving on the batched token hand-off
set -u
mkdir -p gpurun_out/r4s2
for R in open1 closed open2; do
  if [ $R = closed ]; then A="--clients 64 --requests 4"; else A="--rate 140 --num-requests 256 --long-frac 0"; fi
  timeout -k 10 400 python -u bench/serving_bench.py --model gpt2-xl $A > gpurun_out/r4s2/$R.log 2>&1 || { tail -60 gpurun_out/r4s2/$R.log; exit 1; }
  echo "$R $(tail -1 gpurun_out/r4s2/$R.log)" | tee -a gpurun_out/r4s2/summary.txt | cut -c1-400
done
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r4s2/bench10.log 2>&1 || { tail -30 gpurun_out/r4s2/bench10.log; exit 1; }
tail -1 gpurun_out/r4s2/bench10.log | cut -c1-300
