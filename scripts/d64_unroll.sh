# decode attention unroll sweep for D = 64 (GPT-2-XL) and D = 128 (Llama-2-7B), HBM-cold scattered pages
mkdir -p gpurun_out/unroll
timeout -k 10 200 python bench/attn_bench.py --B 64 --ctx 128,192,256 --heads 25:25 --D 64 --unrolls 1,2,4,11,12,14 --random-pages > gpurun_out/unroll/d64.log 2>&1 || exit $?
timeout -k 10 200 python bench/attn_bench.py --B 64 --ctx 192,256 --heads 32:32 --D 128 --unrolls 1,2,4,11,12,14 --random-pages > gpurun_out/unroll/d128.log 2>&1 || exit $?
grep -h "{" gpurun_out/unroll/*.log | cut -c1-400
