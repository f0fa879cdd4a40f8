# the other BASELINE configs and model families on the final round-6 tree (one MI355X; bench.py shape: 64 requests
# per GPU, 128 + 128 tokens). usage: bash scripts/r6_configs.sh a|b
set -u
O=gpurun_out/r6cfg
mkdir -p $O
run() { local n=$1; shift; timeout -k 10 500 python bench.py "$@" --secondary none > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' $O/$n.log | tr '\n' ' ')"; }
if [ "$1" = a ]; then
run llama7b_tp8sim_comm_tbo --simulate-tp 8 --sim-comm 15,150 --sim-tbo 128 --steps 2 --warmup 1 &&
run llama13b_tp1 --model llama2-13b --steps 2 --warmup 1 &&
run llama13b_tp8sim --model llama2-13b --simulate-tp 8 --steps 2 --warmup 1 &&
run llama13b_tp8sim_comm_tbo --model llama2-13b --simulate-tp 8 --sim-comm 15,150 --sim-tbo 128 --steps 2 --warmup 1
else
run gptj6b_tp1 --model gptj-6b --steps 2 --warmup 1 &&
run santacoder_tp1 --model santacoder --steps 2 --warmup 1 &&
run starcoder_tp1 --model starcoder --steps 2 --warmup 1 &&
run llama70b_fp8_tp1 --model llama2-70b --fp8 --steps 2 --warmup 1
fi
