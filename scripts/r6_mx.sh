# round 6: the MX-fp8 SwiGLU -> down hand-off (gemm_mid MXA) - kernel + model tests, the Llama-2-70B fp8 TP=8 shard
# bench, and its decode window (rocprofv3 kernel trace)
set -u
mkdir -p gpurun_out/r6mx
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_kernels_gpu.py -k "mx_output or w8a8_mid or w8a8_mx" \
  tests/test_hf_parity_gpu.py -k "w8a8 or mx_handoff" -s > gpurun_out/r6mx/tests.log 2>&1 || { tail -40 gpurun_out/r6mx/tests.log; exit 1; }
tail -3 gpurun_out/r6mx/tests.log; grep -E "MX hand-off|per-GEMM|W8A8 GPU" gpurun_out/r6mx/tests.log
timeout -k 10 600 python3 bench.py --model llama2-70b --fp8 --simulate-tp 8 --secondary none --steps 2 --warmup 1 \
  > gpurun_out/r6mx/llama70b_fp8_tp8sim.log 2>&1 || { tail -20 gpurun_out/r6mx/llama70b_fp8_tp8sim.log; exit 1; }
grep -E "autotuned|engine ready" gpurun_out/r6mx/llama70b_fp8_tp8sim.log; tail -1 gpurun_out/r6mx/llama70b_fp8_tp8sim.log | cut -c1-300
BENCH_ARGS="--model llama2-70b --fp8 --simulate-tp 8 --secondary none --steps 2 --warmup 1" ANCHOR=sample_v3 SKIP=0.6 SPAN=16000 bash scripts/tp1_trace.sh || exit $?
python3 scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r6mx/llama70b_fp8_tp8sim_window.summary.txt
rm -f gpurun_out/tp1_window.csv
head -16 gpurun_out/r6mx/llama70b_fp8_tp8sim_window.summary.txt
