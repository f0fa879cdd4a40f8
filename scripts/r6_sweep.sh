# round 6: prompt-batch GEMM plans on GPT-2-XL / Llama-2-7B shapes at M = 8192
set -u
mkdir -p gpurun_out/r6s
for m in gpt2-xl llama2-7b; do
  timeout -k 10 300 python3 -u bench/prefill_sweep.py --model $m > gpurun_out/r6s/sweep_$m.log 2>&1 || { tail -20 gpurun_out/r6s/sweep_$m.log; exit 1; }
done
