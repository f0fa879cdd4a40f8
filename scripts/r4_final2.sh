# round 4 last pass on the final tree: GPU suite, smoke, bench; then the GPT-2-XL GEMM probe
set -u
mkdir -p gpurun_out/r4f2
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r4f2/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4f2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4f2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f2/smoke.log 2>&1 || { tail -20 gpurun_out/r4f2/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r4f2/bench.log 2>&1 || { tail -20 gpurun_out/r4f2/bench.log; exit 1; }
tail -1 gpurun_out/r4f2/bench.log | cut -c1-200
if [ -x ./bench/proto/midm_probe ]; then timeout -k 10 300 ./bench/proto/midm_probe gpt2 > gpurun_out/r4f2/midm_gpt2.log 2>&1; fi
