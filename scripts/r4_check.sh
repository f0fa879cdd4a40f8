#!/bin/bash
# round 4: GPU tests touched this round + TP=8-shard sims (all-reduce vs row-sharded schedule) + M=64 GEMM sweep
set -u
mkdir -p gpurun_out/r4
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/r4/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/r4/$name.log"; return $rc; }
run tests 500 python -u -m pytest tests/test_comm_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -x -q --timeout 240 --timeout-method thread || exit $?
run sim8 240 python bench.py --simulate-tp 8 --steps 3 --warmup 1 --sim-comm 15,150 || exit $?
LLMSS_TP_RSAG=1 run sim8_rsag 240 python bench.py --simulate-tp 8 --steps 3 --warmup 1 --sim-comm 15,150 || exit $?
run sweep64 300 python -u bench/tp8_gemm_sweep.py --m 64 --tp1 --deep --top 8 || exit $?
