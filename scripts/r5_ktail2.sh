# round 5: K-tail as a template parameter (the K % 64 == 0 kernel compiles as before): GEMM tests, headline bench x2
set -u
mkdir -p gpurun_out/r5kt2
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "gemm_big_edges or gemm_tiled_variants" > gpurun_out/r5kt2/tests.log 2>&1 || { tail -30 gpurun_out/r5kt2/tests.log; exit 1; }
tail -1 gpurun_out/r5kt2/tests.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --secondary none > gpurun_out/r5kt2/bench$i.log 2>&1 || { tail -30 gpurun_out/r5kt2/bench$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5kt2/bench$i.log').read().strip().splitlines()[-1]); print('bench$i', d['value'], d['p50_tpot_ms'], d['p50_ttft_ms'])"
done
timeout -k 10 300 python bench/pp_probe.py --vars "" --shapes qkv,o,gate_up,down --rounds 3 > gpurun_out/r5kt2/pp_probe.jsonl 2>&1 || exit 1
grep -v amdgpu gpurun_out/r5kt2/pp_probe.jsonl | cut -c1-160
