# GPU: W8A8 kernel tests (incl. the gemm_mid fp8 tiles), then Llama-2-70B fp8 TP=1 and TP=8-shard benches
mkdir -p gpurun_out/fp8
T="--timeout 120 --timeout-method thread"
timeout -k 10 600 python -u -m pytest -x -q $T tests/test_kernels_gpu.py -k "w8a8 or fp8 or test_native_loaded or streaming_kernels" > gpurun_out/fp8/kernels.log 2>&1 &&
timeout -k 10 900 python bench.py --model llama2-70b --fp8 --steps 2 --warmup 1 --secondary none > gpurun_out/fp8/llama70b_fp8_tp1.log 2>&1 &&
timeout -k 10 900 python bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/fp8/llama70b_fp8_tp8sim.log 2>&1
rc=$?; for f in gpurun_out/fp8/*.log; do echo "== $f"; tail -n 2 $f | cut -c1-600; done; exit $rc
