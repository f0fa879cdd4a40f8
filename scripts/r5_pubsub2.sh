# round 5: pub/sub serving with the front-end + broker in their own process (as a producer server and Redis would
# be) vs in the engine process vs direct gRPC
set -u
mkdir -p gpurun_out/r5ps
run() {
  timeout -k 10 500 python bench/serving_bench.py "$@" > gpurun_out/r5ps/$TAG.log 2>&1 || { tail -30 gpurun_out/r5ps/$TAG.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ps/$TAG.log').read().strip().splitlines()[-1]); e=d['engine_stats']; print('$TAG', d['value'], d['p50_ttft_ms'], 'steps', e['steps'], 'prefill', e['prefill_steps'])"
}
TAG=own_gpt2-xl_pubsub run --model gpt2-xl --mode pubsub
TAG=inproc_gpt2-xl_pubsub run --model gpt2-xl --mode pubsub --frontend-inproc
TAG=own_gpt2-xl_grpc run --model gpt2-xl --mode grpc
TAG=own_llama2-13b_pubsub run --model llama2-13b --mode pubsub
