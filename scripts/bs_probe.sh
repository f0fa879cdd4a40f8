mkdir -p gpurun_out/bs
for bs in 16 32 64; do
  timeout -k 10 120 python bench/attn_bench.py --B 64 --ctx 192,256 --heads 32:32 --D 128 --unrolls 0 --bs $bs --random-pages >> gpurun_out/bs/llama_d128.log 2>&1 || exit $?
  timeout -k 10 120 python bench/attn_bench.py --B 64 --ctx 192,256 --heads 25:25 --D 64 --unrolls 0 --bs $bs --random-pages >> gpurun_out/bs/gpt2_d64.log 2>&1 || exit $?
done
grep -h "{" gpurun_out/bs/*.log | cut -c1-300
