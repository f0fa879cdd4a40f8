# round 6: Llama-2-70B fp8 TP=8 shard (simulated, no comm) with the W8A8_ILV candidates in the autotuner
set -u
mkdir -p gpurun_out/r6f8
timeout -k 10 600 python3 bench.py --model llama2-70b --fp8 --simulate-tp 8 --secondary none --steps 2 --warmup 1 \
  > gpurun_out/r6f8/llama70b_fp8_tp8sim.log 2>&1 || { tail -20 gpurun_out/r6f8/llama70b_fp8_tp8sim.log; exit 1; }
grep -E "autotuned|engine ready" gpurun_out/r6f8/llama70b_fp8_tp8sim.log; tail -1 gpurun_out/r6f8/llama70b_fp8_tp8sim.log | cut -c1-400
