set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export LLMSS_AUTOTUNE=0
for mode in on off; do
  if [ $mode = off ]; then export LLMSS_TP_DECODE_OVERLAP_MIN=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tbo_tr_$mode -o run --output-format csv -- python3 bench.py --simulate-tp 8 --sim-comm ${SIM:-0.1,100000} --steps 1 --warmup 0 > gpurun_out/tbo_tr_$mode.log 2>&1
  python scripts/trace_window.py gpurun_out/tbo_tr_$mode/run_kernel_trace.csv gpurun_out/tbo_window_$mode.csv --span-us 12000
  rm -f gpurun_out/tbo_tr_$mode/*kernel_trace.csv
done
