#!/bin/bash
# gemm_big K-loop schedule A/B: numerics of every schedule, then M=2048/8192 timings vs hipBLASLt
set -u
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_big_schedules or (test_gemm_tiled_variants and tile4)" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/big_tests.log 2>&1 || { tail -30 gpurun_out/r4/big_tests.log; exit 1; }
tail -2 gpurun_out/r4/big_tests.log
timeout -k 10 400 python bench/gemm_bench.py --m 2048,8192 --big-sched 0,1,2 > gpurun_out/r4/big_ab.log 2>&1 || { tail -20 gpurun_out/r4/big_ab.log; exit 1; }
