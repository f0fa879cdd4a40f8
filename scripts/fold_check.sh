mkdir -p gpurun_out/fold
T="--timeout 120 --timeout-method thread"
timeout -k 10 600 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "norm_fold or test_native_loaded or qkv_gemm_rope_cache_epilogue" > gpurun_out/fold/kernels.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q $T tests/test_engine_gpu.py > gpurun_out/fold/engine.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/fold/bench_fold.log 2>&1 &&
LLMSS_NORM_FOLD=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/fold/bench_nofold.log 2>&1
rc=$?; tail -3 gpurun_out/fold/*.log; exit $rc
