#!/bin/bash
# round 4: kernel numerics + GEMM bench + bench + GPU tests touched this round + TP=8 sims
set -u
mkdir -p gpurun_out/r4
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/r4/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/r4/$name.log"; return $rc; }
run kernels 420 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread || exit $?
run gemm_epi 300 python bench/gemm_bench.py --m 64,8192 || exit $?
run bench 400 python bench.py || exit $?
run tests 600 python -u -m pytest tests/test_comm_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread || exit $?
run sim8 240 python bench.py --simulate-tp 8 --steps 3 --warmup 1 --sim-comm 15,150 || exit $?
LLMSS_TP_RSAG=1 run sim8_rsag 240 python bench.py --simulate-tp 8 --steps 3 --warmup 1 --sim-comm 15,150 || exit $?
