# round 6: in-situ decode GEMM plan A/B for Llama-2-7B TP=1 (o / down / qkv plans forced vs tuned)
set -u
mkdir -p gpurun_out/r6i
timeout -k 10 900 python3 -u bench/insitu_ab.py --model llama2-7b > gpurun_out/r6i/insitu_llama2-7b.log 2>&1 || { tail -20 gpurun_out/r6i/insitu_llama2-7b.log; exit 1; }
grep variant gpurun_out/r6i/insitu_llama2-7b.log
