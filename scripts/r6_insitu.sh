# round 6: in-situ decode GEMM plan A/B (GPT-2-XL) + the pub/sub bench after the broker / front-end rewrite
set -u
mkdir -p gpurun_out/r6i
timeout -k 10 500 python3 -u bench/insitu_ab.py --model gpt2-xl > gpurun_out/r6i/insitu_gpt2-xl.log 2>&1 || { tail -20 gpurun_out/r6i/insitu_gpt2-xl.log; exit 1; }
grep variant gpurun_out/r6i/insitu_gpt2-xl.log
