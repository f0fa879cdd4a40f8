# round 5: fused-QKV decode attention, prologue after the first K/V loads: kernel tests, bench A/B, decode windows
set -u
mkdir -p gpurun_out/r5fq
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "attn_decode" > gpurun_out/r5fq/tests4.log 2>&1 || { tail -40 gpurun_out/r5fq/tests4.log; exit 1; }
tail -1 gpurun_out/r5fq/tests4.log
for e in 1 0; do
  LLMSS_DECODE_FQ=$e timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r5fq/bench4_fq$e.log 2>&1 || { tail -20 gpurun_out/r5fq/bench4_fq$e.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5fq/bench4_fq$e.log').read().strip().splitlines()[-1]); s=d.get('secondary',{}); print('fq=$e', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'], 'gpt2xl', s.get('value'), s.get('p50_tpot_ms'))"
done
for e in 1 0; do
  LLMSS_DECODE_FQ=$e BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
  python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r5fq/llama7b_window4_fq$e.summary.txt
  rm -f gpurun_out/tp1_window.csv
  head -12 gpurun_out/r5fq/llama7b_window4_fq$e.summary.txt
done
