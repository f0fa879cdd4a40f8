# kernel statistics of the headline bench (Llama-2-7B TP=1 + the served GPT-2-XL secondary) on the final round-6
# tree, then the steady-state decode windows of both models (scripts/r6_windows.sh)
set -u
mkdir -p gpurun_out/r6zp
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r6zp/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r6zp/bench.log 2>&1 || { tail -30 gpurun_out/r6zp/bench.log; exit 1; }
tail -1 gpurun_out/r6zp/bench.log | cut -c1-300
find gpurun_out/r6zp/prof -name "*kernel_trace.csv" -delete
find gpurun_out/r6zp/prof -name "*.csv"
bash scripts/r6_windows.sh
