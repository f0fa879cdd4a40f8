# round 6: pub/sub vs direct gRPC serving on GPT-2-XL after the re-submission-aware admission window
# (serving/driver.py _collect: expected re-submissions, near-drain hold); engine_stats carry admit_steps
set -u
mkdir -p gpurun_out/r6p
for mode in grpc pubsub; do
  timeout -k 10 420 python3 bench/serving_bench.py --model gpt2-xl --mode $mode > gpurun_out/r6p/gpt2-xl_$mode.log 2>&1 \
    || { tail -30 gpurun_out/r6p/gpt2-xl_$mode.log; exit 1; }
  tail -3 gpurun_out/r6p/gpt2-xl_$mode.log
done
