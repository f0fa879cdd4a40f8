#!/bin/bash
# PMC passes for the non-GEMM hot kernels (own runs: --pmc with --kernel-trace only, one pass per run).
# usage: scripts/pmc_kernels.sh OUTDIR decode prefill sample add_norm rope
set -u
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA"
i=0
for k in "$@"; do
  i=$((i+1))
  for p in 1 2 3; do
    eval "PMC=\$P$p"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $PMC -d "$out/c${i}_p$p" -o pmc --output-format csv -- \
      python3 bench/kernel_one.py $k --iters 100 > "$out/c${i}_p$p.log" 2>&1 \
      || { echo "pmc kernel $k pass $p failed rc=$?"; exit 1; }
  done
  echo "c$i: $k" >> "$out/configs.txt"
done
