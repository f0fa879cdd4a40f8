set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tp1_tr -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:-} > gpurun_out/tp1_tr.log 2>&1
python scripts/trace_window.py gpurun_out/tp1_tr/run_kernel_trace.csv gpurun_out/tp1_window.csv --skip-frac ${SKIP:-0.8} --anchor "${ANCHOR:-}" --span-us ${SPAN:-10000}
rm -f gpurun_out/tp1_tr/*kernel_trace.csv
