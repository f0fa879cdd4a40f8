# round 5: gemm_pp with a partial last K-tile (Llama-2-7B TP=8 down, K = 1376): kernel tests, TP=8 shard sims
set -u
mkdir -p gpurun_out/r5kt
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -rf $T -k "gemm_big_edges or gemm_tiled_variants" > gpurun_out/r5kt/tests.log 2>&1 || { tail -30 gpurun_out/r5kt/tests.log; exit 1; }
tail -1 gpurun_out/r5kt/tests.log
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" --secondary none > gpurun_out/r5kt/$n.log 2>&1 || { tail -20 gpurun_out/r5kt/$n.log; exit 1; }; echo "$n $(grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' gpurun_out/r5kt/$n.log | tr '\n' ' ')"; }
run llama7b_tp8sim --simulate-tp 8 --steps 2 --warmup 1 &&
LLMSS_TP_DECODE_OVERLAP_MIN=128 run llama7b_tp8sim_comm_tbo --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1
