# does the interleaved ring help the TP=1 decode GEMMs (M <= 64)? bench with its candidates from M = 32
set -u
mkdir -p gpurun_out/r4w
LLMSS_MID_ILV_MIN_M=32 timeout -k 10 400 python bench.py > gpurun_out/r4w/bench_ilv32.log 2>&1 || { tail -20 gpurun_out/r4w/bench_ilv32.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r4w/bench_ilv128.log 2>&1 || { tail -20 gpurun_out/r4w/bench_ilv128.log; exit 1; }
bash scripts/r4_windows.sh
