mkdir -p gpurun_out/serving
for mode in grpc pubsub; do
  timeout -k 10 300 python bench/serving_bench.py --model gpt2-xl --mode $mode > gpurun_out/serving/$mode.log 2>&1 || { tail -30 gpurun_out/serving/$mode.log; exit 1; }
  tail -1 gpurun_out/serving/$mode.log | cut -c1-300
done
timeout -k 10 300 python bench.py --model gpt2-xl > gpurun_out/serving/gpt2xl_bench.log 2>&1 && tail -1 gpurun_out/serving/gpt2xl_bench.log | cut -c1-300
