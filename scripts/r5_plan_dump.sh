# round 5: every decode GEMM candidate of the Llama-2-7B TP=1 shapes at M = 64 (bench/plan_dump.py)
set -u
mkdir -p gpurun_out/r5pd
for shp in "64 12288 4096 --partial" "64 4096 4096 --partial" "64 22016 4096 --glu" "64 4096 11008 --partial"; do
  timeout -k 10 300 python bench/plan_dump.py $shp --top 25 >> gpurun_out/r5pd/tp1.log 2>&1 || { tail -20 gpurun_out/r5pd/tp1.log; exit 1; }
done
cat gpurun_out/r5pd/tp1.log
