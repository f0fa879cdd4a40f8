# GPU: GEMM tile tests, the driver-shaped bench, and the TP=8 shard of the 8-GPU config (batch 512, no comm)
mkdir -p gpurun_out/t7
T="--timeout 120 --timeout-method thread"
timeout -k 10 900 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "tiled_variants or combine_in_launch or norm_fold or w8a8_mid or test_native_loaded or qkv_gemm_rope" > gpurun_out/t7/kernels.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/t7/bench.log 2>&1 &&
timeout -k 10 600 python bench.py --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/t7/tp8sim.log 2>&1
rc=$?; for f in gpurun_out/t7/*.log; do echo "== $f"; tail -n 2 $f | cut -c1-300; done; grep -h autotuned gpurun_out/t7/*.log | cut -c1-400; exit $rc
