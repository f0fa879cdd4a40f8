# GPU: GEMM tile tests incl. the 64x32 gemm_mid tile, then the driver-shaped bench (GPT-2-XL secondary)
mkdir -p gpurun_out/t14
T="--timeout 120 --timeout-method thread"
timeout -k 10 900 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "tiled_variants or combine_in_launch or norm_fold or w8a8_mid or test_native_loaded" > gpurun_out/t14/kernels.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/t14/bench.log 2>&1
rc=$?; for f in gpurun_out/t14/*.log; do echo "== $f"; tail -n 2 $f | cut -c1-300; done; exit $rc
