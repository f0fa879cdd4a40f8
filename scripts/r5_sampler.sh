# round 5: sampler boundary-bin selection by bitonic sort instead of all-pairs ranks: tests, then the sampler bench
set -u
mkdir -p gpurun_out/r5smp
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_dist_sampler.py -q -x -rf $T -k "sample or cand" > gpurun_out/r5smp/tests.log 2>&1 || { tail -40 gpurun_out/r5smp/tests.log; exit 1; }
tail -1 gpurun_out/r5smp/tests.log
timeout -k 10 150 python bench/sampler_bench.py > gpurun_out/r5smp/after.jsonl && cut -c1-100 gpurun_out/r5smp/after.jsonl
