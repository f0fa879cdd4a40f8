# round 4 closing check after the serving changes: GPU suite, smoke
set -u
mkdir -p gpurun_out/r4f4
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r4f4/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4f4/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4f4/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f4/smoke.log 2>&1 || { tail -20 gpurun_out/r4f4/smoke.log; exit 1; }
