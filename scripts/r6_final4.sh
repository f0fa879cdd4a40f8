# round 6 (last): GPU suite + smoke, driver-shaped bench (N=1) and the simulated TP=8 shard on the final tree
# (setup time of the two-round autotuning, shard throughput)
set -u
mkdir -p gpurun_out/r6z4
T="--timeout 300 --timeout-method thread"
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x -rf $T > gpurun_out/r6z4/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6z4/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6z4/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z4/smoke.log 2>&1 || { tail -20 gpurun_out/r6z4/smoke.log; exit 1; }
tail -1 gpurun_out/r6z4/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6z4/bench.json 2> gpurun_out/r6z4/bench.err || { tail -30 gpurun_out/r6z4/bench.err; exit 1; }
cut -c1-400 gpurun_out/r6z4/bench.json
timeout -k 10 600 python bench.py --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/r6z4/tp8sim.json 2> gpurun_out/r6z4/tp8sim.err || { tail -30 gpurun_out/r6z4/tp8sim.err; exit 1; }
cut -c1-400 gpurun_out/r6z4/tp8sim.json
