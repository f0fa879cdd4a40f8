# kernel stats of the simulated TP=8 shard with the column-chunked schedule (why is it slow?)
set -u
mkdir -p gpurun_out/r5c
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LLMSS_TP_COL=4 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c/prof -o run --output-format csv -- python3 bench.py --simulate-tp 8 --sim-comm 15,150 --steps 1 --warmup 1 --secondary none > gpurun_out/r5c/prof.log 2>&1 || { tail -20 gpurun_out/r5c/prof.log; exit 1; }
rm -f gpurun_out/r5c/prof/*kernel_trace.csv
head -25 gpurun_out/r5c/prof/run_kernel_stats.csv | cut -c1-220
