# round 5: prompt-batch QKV projection with the RoPE + KV-write epilogue on the ping-pong kernel: tests, bench,
# prefill-step trace
set -u
mkdir -p gpurun_out/r5pe
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "qkv_prompt_batch_epilogue or qkv_gemm_rope_cache_epilogue or gemm_big_edges" > gpurun_out/r5pe/tests.log 2>&1 || { tail -40 gpurun_out/r5pe/tests.log; exit 1; }
tail -1 gpurun_out/r5pe/tests.log
timeout -k 10 900 python -u -m pytest tests/test_hf_parity_gpu.py tests/test_engine_gpu.py tests/test_chunked_prefill.py tests/test_tp_gpu.py -q -x -rf $T > gpurun_out/r5pe/parity.log 2>&1 || { tail -40 gpurun_out/r5pe/parity.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5pe/parity.log | tail -1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r5pe/bench.log 2>&1 || { tail -20 gpurun_out/r5pe/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r5pe/bench.log').read().strip().splitlines()[-1]); s=d.get('secondary',{}); print('bench', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'], 'gpt2xl', s.get('value'), s.get('p50_ttft_ms'))"
sed -i 's#gpurun_out/r5pt#gpurun_out/r5pe/pt#g' scripts/r5_prefill_trace.sh
bash scripts/r5_prefill_trace.sh | head -8
