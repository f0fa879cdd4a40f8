# round 6: two kv heads per workgroup for D = 64 MHA decode attention (GPT-2-XL) - tests, microbench, bench
set -u
mkdir -p gpurun_out/r6ap
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode" > gpurun_out/r6ap/tests.log 2>&1 || { tail -30 gpurun_out/r6ap/tests.log; exit 1; }
tail -1 gpurun_out/r6ap/tests.log
timeout -k 10 300 python3 bench/attn_bench.py --D 64 --heads 25:25,12:12 --ctx 192,1024 --unrolls 11 --pairs 0,1 \
  > gpurun_out/r6ap/attn_bench.log 2>&1 || { tail -20 gpurun_out/r6ap/attn_bench.log; exit 1; }
cat gpurun_out/r6ap/attn_bench.log | grep "{"
timeout -k 10 600 python3 bench.py --model gpt2-xl --secondary none --steps 10 --warmup 3 > gpurun_out/r6ap/bench.json 2> gpurun_out/r6ap/bench.err || { tail -20 gpurun_out/r6ap/bench.err; exit 1; }
cut -c1-200 gpurun_out/r6ap/bench.json; grep -o '"p50_tpot_ms": [0-9.]*' gpurun_out/r6ap/bench.json
