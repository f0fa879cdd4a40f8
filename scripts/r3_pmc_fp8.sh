# PMC of the W8A8 GEMM at M=64 on the 70B TP=1 QKV shape (N=10240, K=8192): gemm_mid fp8 tile 64x128 (tile 11)
# vs the older gemm_f8f8 64x128 kernel (tile 2), split 3 each
set -u
out=gpurun_out/pmc_fp8
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA"
i=0
for cfg in "11,3" "2,3"; do
  i=$((i+1))
  for p in 1 2 3; do
    eval "PMC=\$P$p"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $PMC -d "$out/c${i}_p$p" -o pmc --output-format csv -- \
      python3 bench/gemm_one.py --m 64 --n 10240 --k 8192 --w8a8 $cfg --split 3 --iters 100 > "$out/c${i}_p$p.log" 2>&1 \
      || { echo "pmc cfg $i pass $p failed rc=$?"; exit 1; }
  done
  echo "c$i: 64 10240 8192 w8a8 $cfg split 3" >> "$out/configs.txt"
done
python scripts/pmc_table.py $out --match "gemm_mid|gemm_f8f8" > $out/table.json
find $out -name '*kernel_trace.csv' -delete
cat $out/table.json | head -60; grep -h 'TB/s' $out/c*_p1.log
