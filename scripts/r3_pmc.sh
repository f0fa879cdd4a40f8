# round 3 PMC: the new gemm_mid tiles vs the plans they replaced (Llama-2-7B QKV at M=64: 64x192 vs 64x128;
# GPT-2-XL MLP up at M=64: 64x32 unsplit vs 64x64 split 2)
bash scripts/pmc_gemm_cfgs.sh gpurun_out/pmc_r3 "64 12288 4096 0x1d00 3" "64 12288 4096 0x2b00 2" \
  "64 6400 1600 0x2e00 1" "64 6400 1600 0x2300 2" || exit $?
python scripts/pmc_table.py gpurun_out/pmc_r3 --match "gemm_mid|gemm_tiled" > gpurun_out/pmc_r3/table.json
find gpurun_out/pmc_r3 -name '*kernel_trace.csv' -delete
cat gpurun_out/pmc_r3/table.json | head -80
