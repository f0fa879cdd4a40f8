# GPU: GEMM kernel tests for the tiled / mid / fold paths, engine tests, then the driver-shaped bench
mkdir -p gpurun_out/tile
T="--timeout 120 --timeout-method thread"
timeout -k 10 900 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "norm_fold or tiled_variants or combine_in_launch or test_native_loaded" > gpurun_out/tile/kernels.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q $T tests/test_engine_gpu.py > gpurun_out/tile/engine.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/tile/bench.log 2>&1
rc=$?; for f in gpurun_out/tile/*.log; do echo "== $f"; tail -n 3 $f; done; exit $rc
