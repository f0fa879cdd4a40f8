# round 5: decode attention fed by the QKV GEMM's output (RoPE + KV write in the attention prologue):
# kernel tests, model parity / engine GPU tests, then the headline bench with and without it
set -u
mkdir -p gpurun_out/r5fq
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "attn_decode or rope_cache" > gpurun_out/r5fq/tests.log 2>&1 || { tail -40 gpurun_out/r5fq/tests.log; exit 1; }
tail -1 gpurun_out/r5fq/tests.log
timeout -k 10 900 python -u -m pytest tests/test_hf_parity_gpu.py tests/test_engine_gpu.py tests/test_chunked_prefill.py tests/test_kv_fp8.py -q -x -rf $T > gpurun_out/r5fq/parity.log 2>&1 || { tail -40 gpurun_out/r5fq/parity.log; exit 1; }
tail -1 gpurun_out/r5fq/parity.log
for e in 1 0; do
  LLMSS_DECODE_FQ=$e timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r5fq/bench_fq$e.log 2>&1 || { tail -20 gpurun_out/r5fq/bench_fq$e.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5fq/bench_fq$e.log').read().strip().splitlines()[-1]); s=d.get('secondary',{}); print('fq=$e', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'], 'gpt2xl', s.get('engine_direct_tokens_per_s', s.get('value')), s.get('p50_tpot_ms'))"
done
