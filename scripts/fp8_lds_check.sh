# fp8 fragment chunks g / g+4 (conflict-free): W8A8 kernel tests, PMC of the fp8 gemm_mid tile, 70B fp8 TP=1 bench
mkdir -p gpurun_out/f8lds
T="--timeout 120 --timeout-method thread"
timeout -k 10 600 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "w8a8 or fp8 or test_native_loaded" > gpurun_out/f8lds/kernels.log 2>&1 || exit $?
rm -rf gpurun_out/pmc_fp8 && bash scripts/r3_pmc_fp8.sh > gpurun_out/f8lds/pmc.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --model llama2-70b --fp8 --steps 2 --warmup 1 --secondary none > gpurun_out/f8lds/llama70b_fp8_tp1.log 2>&1 || exit $?
tail -n 2 gpurun_out/f8lds/kernels.log; grep -h autotuned gpurun_out/f8lds/llama70b_fp8_tp1.log | cut -c1-400
grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*' gpurun_out/f8lds/llama70b_fp8_tp1.log
