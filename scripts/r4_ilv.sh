# round 4: gemm_mid interleaved ring (numerics, TP=8 shard sweep), decode twins (numerics, bench A/B)
set -u
mkdir -p gpurun_out/r4w
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "twin or packed" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4w/twin_tests.log 2>&1 || { tail -30 gpurun_out/r4w/twin_tests.log; exit 1; }
tail -1 gpurun_out/r4w/twin_tests.log
LLMSS_DECODE_TWIN=qkv,up timeout -k 10 400 python bench.py > gpurun_out/r4w/bench_twin.log 2>&1 || { tail -20 gpurun_out/r4w/bench_twin.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r4w/bench_notwin.log 2>&1 || { tail -20 gpurun_out/r4w/bench_notwin.log; exit 1; }
