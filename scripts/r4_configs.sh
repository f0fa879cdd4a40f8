# the other BASELINE configs on the final round-4 tree (one MI355X)
set -u
mkdir -p gpurun_out/r4c
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" --secondary none > gpurun_out/r4c/$n.log 2>&1 || { tail -20 gpurun_out/r4c/$n.log; exit 1; }; echo "$n $(grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' gpurun_out/r4c/$n.log | tr '\n' ' ')"; }
run llama7b_tp8sim --simulate-tp 8 --steps 2 --warmup 1
run llama7b_tp8sim_comm --simulate-tp 8 --sim-comm 15,150 --steps 2 --warmup 1
run llama13b_tp1 --model llama2-13b --steps 2 --warmup 1
run llama13b_tp8sim --model llama2-13b --simulate-tp 8 --steps 2 --warmup 1
run llama70b_fp8_tp8sim --model llama2-70b --fp8 --simulate-tp 8 --steps 2 --warmup 1
