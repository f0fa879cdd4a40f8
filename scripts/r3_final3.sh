# round 3 closing check on the final tree: GPU suite, smoke, driver-shaped bench
mkdir -p gpurun_out/final3
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/final3/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/final3/bench.log 2>&1 || exit $?
tail -n 2 gpurun_out/final3/pytest_gpu.log; tail -n 1 gpurun_out/final3/smoke.log | cut -c1-200; tail -n 1 gpurun_out/final3/bench.log | cut -c1-300
