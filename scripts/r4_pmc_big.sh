# counters of the prefill GEMM (gemm_big, 256x256) at M = 8192 on the Llama qkv shape: LDS conflicts after the
# epilogue change, MFMA busy after the interleaved K-loop. Each pass is its own run (--pmc with kernel-trace only).
set -u
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
A="--m 8192 --n 12288 --k 4096 --hint 0x400 --split 1 --iters 20"
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/r4p/p1 -o pmc --output-format csv -- python3 bench/gemm_one.py $A > gpurun_out/r4p/p1.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/r4p/p2 -o pmc --output-format csv -- python3 bench/gemm_one.py $A > gpurun_out/r4p/p2.log 2>&1 || exit 1
rm -f gpurun_out/r4p/*/pmc_kernel_trace.csv
