# served GPT-2-XL over 20 steps with and without the engine's gc.freeze (LLMSS_GC_FREEZE)
set -u
mkdir -p gpurun_out/r4g
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r4g/bench_gcfreeze.log 2>&1 || { tail -20 gpurun_out/r4g/bench_gcfreeze.log; exit 1; }
LLMSS_GC_FREEZE=0 timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r4g/bench_nogcfreeze.log 2>&1 || { tail -20 gpurun_out/r4g/bench_nogcfreeze.log; exit 1; }
