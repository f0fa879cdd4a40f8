# round 6: the many-CU modelled collective - kernel test, then the simulated Llama-2-7B TP=8 shard with one all-reduce
# vs two micro-batches under the one-workgroup spin model (round 5's) and the 32-channel model
set -u
mkdir -p gpurun_out/r6cm
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "comm_model" > gpurun_out/r6cm/tests.log 2>&1 || { tail -30 gpurun_out/r6cm/tests.log; exit 1; }
tail -1 gpurun_out/r6cm/tests.log
run() {
  timeout -k 10 500 python3 bench.py --simulate-tp 8 --secondary none --steps 2 --warmup 1 "$@" > gpurun_out/r6cm/$name.json 2> gpurun_out/r6cm/$name.err \
    || { tail -20 gpurun_out/r6cm/$name.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6cm/$name.json')); print('$name', d['value'], d['p50_tpot_ms'], d['config']['parallelism'])"
}
name=spin_ar run --sim-comm 15,150 && name=spin_tbo run --sim-comm 15,150 --sim-tbo 128 && \
name=ch32_ar run --sim-comm 15,150,32 && name=ch32_tbo run --sim-comm 15,150,32 --sim-tbo 128
