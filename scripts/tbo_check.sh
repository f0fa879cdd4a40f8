set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "microbatch or rccl or overlap" > gpurun_out/tbo_tests.log 2>&1
LLMSS_TP_DECODE_OVERLAP_MIN=0 timeout -k 10 300 python bench.py --simulate-tp 8 --sim-comm 10,100 > gpurun_out/tbo_off.log 2>&1
timeout -k 10 300 python bench.py --simulate-tp 8 --sim-comm 10,100 > gpurun_out/tbo_on.log 2>&1
timeout -k 10 300 python bench.py --simulate-tp 8 --sim-comm 0.1,100000 > gpurun_out/tbo_nocomm.log 2>&1
