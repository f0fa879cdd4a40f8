# round 6: Llama-2-13B TP=1 pub/sub vs direct gRPC after the asyncio broker / front-end (config #4's serving path)
set -u
mkdir -p gpurun_out/r6p
for mode in grpc pubsub; do
  timeout -k 10 500 python3 bench/serving_bench.py --model llama2-13b --mode $mode > gpurun_out/r6p/llama2-13b_$mode.log 2>&1 \
    || { tail -30 gpurun_out/r6p/llama2-13b_$mode.log; exit 1; }
  tail -1 gpurun_out/r6p/llama2-13b_$mode.log | cut -c1-330
done
