# GPU: extend-attention tests (chunked prefill + GQA decode through the extend kernel), then 70B fp8 TP=1 / TP=8 shard
mkdir -p gpurun_out/gqa
T="--timeout 120 --timeout-method thread"
timeout -k 10 600 python -u -m pytest -x -q $T tests -m gpu -k "extend or chunked or gqa or kv_fp8 or test_native_loaded" > gpurun_out/gqa/tests.log 2>&1 &&
timeout -k 10 900 python bench.py --model llama2-70b --fp8 --steps 2 --warmup 1 --secondary none > gpurun_out/gqa/llama70b_fp8_tp1.log 2>&1 &&
timeout -k 10 900 python bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/gqa/llama70b_fp8_tp8sim.log 2>&1
rc=$?; for f in gpurun_out/gqa/*.log; do echo "== $f"; tail -n 2 $f | cut -c1-400; done; exit $rc
