# round 6: the software-pipelined fp8 gemm_mid k-loop - kernel tests, then the 70B fp8 TP=8 shard shape probe
set -u
mkdir -p gpurun_out/r6f8
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "w8a8_mid_tiles" > gpurun_out/r6f8/tests.log 2>&1 || { tail -30 gpurun_out/r6f8/tests.log; exit 1; }
tail -2 gpurun_out/r6f8/tests.log
timeout -k 10 400 ./bench/proto/f8_probe > gpurun_out/r6f8/probe.log 2>&1 || { tail -20 gpurun_out/r6f8/probe.log; exit 1; }
grep -c identical gpurun_out/r6f8/probe.log; grep -c DIFFER gpurun_out/r6f8/probe.log || true
