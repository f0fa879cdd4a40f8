# round 5: served throughput through the pub/sub path (gRPC front-end -> RESP broker -> consumer -> engine) vs direct gRPC
set -u
mkdir -p gpurun_out/r5ps
for cfg in "gpt2-xl pubsub" "gpt2-xl grpc" "llama2-13b pubsub" "llama2-13b grpc"; do
  set -- $cfg
  timeout -k 10 500 python bench/serving_bench.py --model $1 --mode $2 > gpurun_out/r5ps/after_$1_$2.log 2>&1 || { tail -30 gpurun_out/r5ps/after_$1_$2.log; exit 1; }
  echo "$1 $2: $(tail -1 gpurun_out/r5ps/after_$1_$2.log | cut -c1-400)"
done
