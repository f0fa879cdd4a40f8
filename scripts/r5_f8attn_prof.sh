# round 5: kernel stats of the 70B fp8 TP=8 shard with the fused attention fp8 twin (is quant_fp8_act<1> gone from decode?)
set -u
mkdir -p gpurun_out/r5fa
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r5fa/prof -o run --output-format csv -- python3 bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 1 --warmup 1 --secondary none > gpurun_out/r5fa/prof.log 2>&1 || { tail -20 gpurun_out/r5fa/prof.log; exit 1; }
find gpurun_out/r5fa/prof -name "*kernel_trace.csv" -delete
grep -h "quant_fp8\|attn_extend" gpurun_out/r5fa/prof/run_kernel_stats.csv | cut -c1-160
