# the other BASELINE configs on the final round-3 tree (one MI355X)
mkdir -p gpurun_out/configs
timeout -k 10 600 python bench.py --model llama2-13b --steps 2 --warmup 1 --secondary none > gpurun_out/configs/llama13b_tp1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --model llama2-13b --simulate-tp 8 --steps 2 --warmup 1 --secondary none > gpurun_out/configs/llama13b_tp8sim.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --batch-per-gpu 256 --steps 2 --warmup 1 --secondary none > gpurun_out/configs/llama7b_b256.log 2>&1 || exit $?
grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' gpurun_out/configs/*.log
