# round 5: the reference's other model families on one MI355X (bench.py shape: 64 requests, 128 + 128 tokens,
# TP=1, bf16 unless noted): GPT-J-6B (rotary, parallel block), SantaCoder and StarCoder (GPT-BigCode MQA),
# and Llama-2-70B with fp8 weights on one GPU
set -u
mkdir -p gpurun_out/r5fam
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" --secondary none > gpurun_out/r5fam/$n.log 2>&1 || { tail -20 gpurun_out/r5fam/$n.log; exit 1; }; echo "$n $(grep -ho '"value": [0-9.]*\|"p50_tpot_ms": [0-9.]*\|"p50_ttft_ms": [0-9.]*' gpurun_out/r5fam/$n.log | tr '\n' ' ')"; }
run gptj6b_tp1 --model gptj-6b --steps 2 --warmup 1 &&
run santacoder_tp1 --model santacoder --steps 2 --warmup 1 &&
run starcoder_tp1 --model starcoder --steps 2 --warmup 1 &&
run llama70b_fp8_tp1 --model llama2-70b --fp8 --steps 2 --warmup 1
