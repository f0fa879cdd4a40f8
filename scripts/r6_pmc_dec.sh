# PMC of the final tree's M = 64 decode GEMM plans (the autotuner's picks in profiles/r6_final2 / gpurun_out/r6z/bench.err)
set -u
O=gpurun_out/r6pmc
bash scripts/pmc_gemm_cfgs.sh $O \
  "64 4800 1600 0x42300 2" "64 1600 1600 0x2e00 5" "64 6400 1600 0x42200 1" "64 1600 6400 0x42200 5" \
  "64 12288 4096 0x42300 1" "64 4096 4096 0x2300 4" "64 4096 11008 0x3300 4" || exit 1
python scripts/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
find $O -name "*.csv" -size +2M -delete
