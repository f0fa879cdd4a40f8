# LDS bank conflicts of the decode GEMM tiles after the epilogue change (M = 64, Llama TP=1 shapes)
set -u
mkdir -p gpurun_out/r4q
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for A in "--m 64 --n 12288 --k 4096 --hint 0x1d00 --split 1" "--m 64 --n 22016 --k 4096 --hint 0x1f00 --split 1 --glu" "--m 64 --n 4096 --k 4096 --hint 0x1b00 --split 2"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/r4q/c$i -o pmc --output-format csv -- python3 bench/gemm_one.py $A --iters 50 > gpurun_out/r4q/c$i.log 2>&1 || exit 1
  echo "c$i: $A" >> gpurun_out/r4q/configs.txt
done
rm -f gpurun_out/r4q/*/pmc_kernel_trace.csv
