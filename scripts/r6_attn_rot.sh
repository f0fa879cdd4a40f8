# decode attention in isolation vs in the decode step (35.5 vs 41.7 us for Llama-2-7B): does a larger rotated
# working set (TLB reach) or scattered pages account for the difference?
set -u
mkdir -p gpurun_out/r6ar
for r in 700 7000 20000; do
  for rp in "" "--random-pages"; do
    echo "rotate_mb=$r $rp" >> gpurun_out/r6ar/attn.log
    timeout -k 10 240 python bench/attn_bench.py --ctx 192 --heads 32:32 --unrolls 0 --rotate-mb $r $rp >> gpurun_out/r6ar/attn.log 2>&1 || exit 1
  done
done
cat gpurun_out/r6ar/attn.log
