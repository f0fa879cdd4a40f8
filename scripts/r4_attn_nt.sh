# decode attention K/V loads: non-temporal (default, unroll 11 / 2) vs default policy (21 / 22); isolated and in-step
set -u
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/tests.log 2>&1 || { tail -30 gpurun_out/r4a/tests.log; exit 1; }
tail -1 gpurun_out/r4a/tests.log
timeout -k 10 200 python bench/attn_bench.py --D 128 --heads 32:32 --ctx 192,256 --unrolls 11,21,2,22 > gpurun_out/r4a/attn_iso.log 2>&1 || exit 1
timeout -k 10 200 python bench/attn_bench.py --D 64 --heads 25:25 --ctx 192 --unrolls 11,21,2,22 >> gpurun_out/r4a/attn_iso.log 2>&1 || exit 1
cat gpurun_out/r4a/attn_iso.log | grep "{"
LLMSS_ATTN_UNROLL=21 timeout -k 10 400 python bench.py > gpurun_out/r4a/bench_21.log 2>&1 || { tail -20 gpurun_out/r4a/bench_21.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r4a/bench_11.log 2>&1 || { tail -20 gpurun_out/r4a/bench_11.log; exit 1; }
