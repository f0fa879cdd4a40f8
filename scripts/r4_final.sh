# round 4 closing evidence on the final tree: GPU suite, smoke, driver-shaped bench, decode windows
set -u
mkdir -p gpurun_out/r4f
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r4f/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4f/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4f/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f/smoke.log 2>&1 || { tail -20 gpurun_out/r4f/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4f/bench.log 2>&1 || { tail -20 gpurun_out/r4f/bench.log; exit 1; }
tail -1 gpurun_out/r4f/bench.log | cut -c1-300
