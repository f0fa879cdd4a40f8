#!/bin/bash
# prompt-batch library routing: numerics, then the headline bench with and without it
set -u
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "library_routing or gemm_big_edges" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/lib_tests.log 2>&1 || { tail -30 gpurun_out/r4/lib_tests.log; exit 1; }
tail -2 gpurun_out/r4/lib_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_lib.log 2>&1 || { tail -20 gpurun_out/r4/bench_lib.log; exit 1; }
grep -h "prompt-batch\|prefill_gemm" gpurun_out/r4/bench_lib.log | cut -c1-400 | head -4
LLMSS_PREFILL_LIB=0 timeout -k 10 400 python bench.py > gpurun_out/r4/bench_nolib.log 2>&1 || { tail -20 gpurun_out/r4/bench_nolib.log; exit 1; }
