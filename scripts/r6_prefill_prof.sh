# round 6: where a GPT-2-XL / Llama-2-7B bench step's device time goes, prefill kernels included (kernel totals over
# the timed steps of a short run under rocprofv3 --kernel-trace)
set -u
mkdir -p gpurun_out/r6g
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in gpt2-xl llama2-7b; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r6g/prof_$m -o run --output-format csv -- python3 bench.py --model $m --secondary none --steps 2 --warmup 1 > gpurun_out/r6g/bench_$m.log 2>&1 || { tail -20 gpurun_out/r6g/bench_$m.log; exit 1; }
  f=$(find gpurun_out/r6g/prof_$m -name "*kernel_trace.csv" | head -1)
  python3 scripts/kernel_totals.py "$f" 40 --bench-log gpurun_out/r6g/bench_$m.log > gpurun_out/r6g/kernels_$m.txt
  rm -f "$f"
  head -14 gpurun_out/r6g/kernels_$m.txt
done
