# round 6: grouped slab loads in add_norm (runtime split counts) and splitk_reduce - kernel tests, then the bench
set -u
mkdir -p gpurun_out/r6s2
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "split_slab or splitk or add_norm or gemm_dec" > gpurun_out/r6s2/tests.log 2>&1 || { tail -30 gpurun_out/r6s2/tests.log; exit 1; }
tail -1 gpurun_out/r6s2/tests.log
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 > gpurun_out/r6s2/bench.json 2> gpurun_out/r6s2/bench.err || { tail -20 gpurun_out/r6s2/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6s2/bench.json')); s=d['secondary']
print('llama', d['value'], d['p50_tpot_ms'], 'gpt2', s['value'], s['p50_tpot_ms'], s['engine_direct']['value'])"
