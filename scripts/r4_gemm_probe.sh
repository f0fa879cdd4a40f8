#!/bin/bash
# round 4: TP=8-shard decode GEMMs (M=512 / 256) - candidate sweep cold and warm, then PMC of chosen plans
set -u
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u bench/tp8_gemm_sweep.py --m 512 --top 6 > gpurun_out/r4/sweep512.log 2>&1 || exit $?
timeout -k 10 300 python -u bench/tp8_gemm_sweep.py --m 512 --top 4 --warm --shapes qkv,up > gpurun_out/r4/sweep512_warm.log 2>&1 || exit $?
timeout -k 10 300 python -u bench/tp8_gemm_sweep.py --m 256 --top 4 > gpurun_out/r4/sweep256.log 2>&1 || exit $?
bash scripts/pmc_gemm_cfgs.sh gpurun_out/r4/pmc "512 1536 4096 0x1300 4" "512 1536 4096 0x1900 8" "512 1536 4096 0x1800 4" "512 1536 4096 0x2800 4" || exit $?
