# round 5 closing check: GPU suite, smoke, headline bench, rocprofv3 kernel stats of the bench process
set -u
mkdir -p gpurun_out/r5f
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r5f/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5f/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5f/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.log 2>&1 || { tail -20 gpurun_out/r5f/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r5f/bench.log 2>&1 || { tail -30 gpurun_out/r5f/bench.log; exit 1; }
tail -1 gpurun_out/r5f/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r5f/bench_prof.log 2>&1 || { tail -30 gpurun_out/r5f/bench_prof.log; exit 1; }
find gpurun_out/r5f/prof -name "*kernel_trace.csv" -delete
find gpurun_out/r5f/prof -name "*kernel_stats.csv" | head -3
