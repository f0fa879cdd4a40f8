# round 5 checkpoint: GPU suite, smoke, headline bench
set -u
mkdir -p gpurun_out/r5k
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r5k/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5k/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5k/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5k/smoke.log 2>&1 || { tail -20 gpurun_out/r5k/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/r5k/bench.log 2>&1 || { tail -30 gpurun_out/r5k/bench.log; exit 1; }
tail -1 gpurun_out/r5k/bench.log | cut -c1-400
