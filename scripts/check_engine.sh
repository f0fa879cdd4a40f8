# engine GPU tests, then the headline bench and the TP=8-shard bench (host pipelining check)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "not sweep" > gpurun_out/ce_tests.log 2>&1 || { tail -30 gpurun_out/ce_tests.log; exit 1; }
tail -1 gpurun_out/ce_tests.log
timeout -k 10 300 python bench.py > gpurun_out/ce_bench.log 2>&1 || { tail -20 gpurun_out/ce_bench.log; exit 1; }
tail -1 gpurun_out/ce_bench.log | cut -c1-330
timeout -k 10 300 python bench.py --simulate-tp 8 > gpurun_out/ce_tp8.log 2>&1 || { tail -20 gpurun_out/ce_tp8.log; exit 1; }
tail -1 gpurun_out/ce_tp8.log | cut -c1-330
