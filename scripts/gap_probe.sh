# keep the decode-window CSVs (TP=1 headline, TP=8 shard) to locate inter-kernel gaps
mkdir -p gpurun_out/gaps
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
cp gpurun_out/tp1_window.csv gpurun_out/gaps/tp1.csv
BENCH_ARGS="--simulate-tp 8 --steps 1 --warmup 1 --secondary none" ANCHOR=sample_cand SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
cp gpurun_out/tp1_window.csv gpurun_out/gaps/tp8.csv
rm -f gpurun_out/tp1_window.csv
