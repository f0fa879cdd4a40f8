# round 5: kernel trace of the simulated TP=8 shard (comm model 15 us + bytes / 150 GB/s), one all-reduce vs two
# micro-batches, comm stream at normal priority: per-stream busy time and overlap in a steady-state decode window
set -u
mkdir -p gpurun_out/r5w
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for cfg in ${CFGS:-one:0 tbo:128}; do
  set -- ${cfg/:/ }
  LLMSS_TP_COL=0 LLMSS_TP_DECODE_OVERLAP_MIN=$2 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5w/tr_$1 -o run --output-format csv -- python3 bench.py --simulate-tp 8 --sim-comm 15,150 --steps 1 --warmup 1 --secondary none > gpurun_out/r5w/$1.log 2>&1 || { tail -20 gpurun_out/r5w/$1.log; exit 1; }
  python scripts/trace_window.py gpurun_out/r5w/tr_$1/run_kernel_trace.csv gpurun_out/r5w/$1_window.csv --skip-frac 0.6 --anchor sample_cand --span-us 12000
  rm -f gpurun_out/r5w/tr_$1/*kernel_trace.csv
  python scripts/stream_overlap.py gpurun_out/r5w/$1_window.csv > gpurun_out/r5w/$1_window.summary.txt
  head -40 gpurun_out/r5w/$1_window.summary.txt
done
