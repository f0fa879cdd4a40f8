# round 5: decode window of the 70B fp8 TP=8 shard with the fused attention fp8 twin
set -u
mkdir -p gpurun_out/r5fa
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r5fa/tr -o run --output-format csv -- python3 bench.py --model llama2-70b --fp8 --simulate-tp 8 --steps 1 --warmup 1 --secondary none > gpurun_out/r5fa/tr.log 2>&1 || { tail -20 gpurun_out/r5fa/tr.log; exit 1; }
python scripts/trace_window.py gpurun_out/r5fa/tr/run_kernel_trace.csv gpurun_out/r5fa/window.csv --skip-frac 0.6 --anchor sample_cand --span-us 20000
rm -f gpurun_out/r5fa/tr/*kernel_trace.csv
python scripts/step_breakdown.py gpurun_out/r5fa/window.csv > gpurun_out/r5fa/window.summary.txt
head -16 gpurun_out/r5fa/window.summary.txt
