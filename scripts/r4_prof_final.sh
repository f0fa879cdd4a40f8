# kernel statistics of the headline bench on the final round-4 tree
set -u
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/r4p/bench.log 2>&1 || { tail -30 gpurun_out/r4p/bench.log; exit 1; }
tail -1 gpurun_out/r4p/bench.log | cut -c1-200
find gpurun_out/r4p/prof -name "*kernel_trace.csv" -delete
find gpurun_out/r4p/prof -name "*.csv" | head
