# round 5: decode attention vs KV page size (tokens per block), cold KV, Llama-2-7B TP=1 and GPT-2-XL heads
set -u
mkdir -p gpurun_out/r5ab
for bs in 16 32 64; do
  timeout -k 10 200 python bench/attn_bench.py --B 64 --ctx 192 --heads 32:32 --D 128 --unrolls 11,12 --bs $bs >> gpurun_out/r5ab/llama.log 2>&1 || exit 1
  timeout -k 10 200 python bench/attn_bench.py --B 64 --ctx 192 --heads 25:25 --D 64 --unrolls 11,12 --bs $bs >> gpurun_out/r5ab/gpt2.log 2>&1 || exit 1
  timeout -k 10 200 python bench/attn_bench.py --B 64 --ctx 192 --heads 32:32 --D 128 --unrolls 11 --bs $bs --random-pages >> gpurun_out/r5ab/llama_rand.log 2>&1 || exit 1
done
grep "{" gpurun_out/r5ab/*.log
