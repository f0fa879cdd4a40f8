# round 5: fp8 QKV GEMM with the RoPE / KV-write epilogue - kernel tests, fp8 parity, 70B fp8 TP=8 shard
set -u
mkdir -p gpurun_out/r5q8
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "qkv_gemm_rope_cache_epilogue" > gpurun_out/r5q8/tests.log 2>&1 || { tail -40 gpurun_out/r5q8/tests.log; exit 1; }
tail -1 gpurun_out/r5q8/tests.log
timeout -k 10 600 python -u -m pytest tests/test_hf_parity_gpu.py tests/test_kv_fp8.py -q -x -rf $T > gpurun_out/r5q8/parity.log 2>&1 || { tail -30 gpurun_out/r5q8/parity.log; exit 1; }
tail -1 gpurun_out/r5q8/parity.log
timeout -k 10 600 python bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/r5q8/llama70b_fp8_tp8sim.log 2>&1 || { tail -20 gpurun_out/r5q8/llama70b_fp8_tp8sim.log; exit 1; }
grep "QKV RoPE" gpurun_out/r5q8/llama70b_fp8_tp8sim.log | cut -c1-400
python3 -c "import json; d=json.loads(open('gpurun_out/r5q8/llama70b_fp8_tp8sim.log').read().strip().splitlines()[-1]); print('70b_fp8_tp8sim', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
