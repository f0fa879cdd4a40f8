mkdir -p gpurun_out/host
LLMSS_HOST_PROFILE=1 timeout -k 10 600 python bench.py --simulate-tp 8 --steps 1 --warmup 1 --secondary none > gpurun_out/host/tp8.log 2>&1 || exit $?
LLMSS_HOST_PROFILE=1 timeout -k 10 400 python bench.py --steps 1 --warmup 1 --secondary none > gpurun_out/host/tp1.log 2>&1 || exit $?
grep -ho '"p50_tpot_ms": [0-9.]*\|"engine_stats": {[^}]*}' gpurun_out/host/tp8.log gpurun_out/host/tp1.log
