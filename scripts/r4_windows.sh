# round 4: decode attention with sequential vs scattered pages, then steady-state decode windows of the
# headline (Llama-2-7B TP=1), GPT-2-XL and the TP=8 shard (batch 512) on the current tree
mkdir -p gpurun_out/r4w
timeout -k 10 200 python bench/attn_bench.py --D 128 --heads 32:32 --ctx 128,192,256 --unrolls 11,2 --random-pages > gpurun_out/r4w/attn_rand.log 2>&1 || exit $?
timeout -k 10 200 python bench/attn_bench.py --D 128 --heads 32:32 --ctx 128,192,256 --unrolls 11,2 > gpurun_out/r4w/attn_seq.log 2>&1 || exit $?
BENCH_ARGS="--steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r4w/llama7b_tp1_window.summary.txt
cp gpurun_out/tp1_window.csv gpurun_out/r4w/llama7b_tp1_window.csv
BENCH_ARGS="--model gpt2-xl --steps 2 --warmup 1 --secondary none" ANCHOR=sample_v3 SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r4w/gpt2xl_window.summary.txt
BENCH_ARGS="--simulate-tp 8 --steps 1 --warmup 1 --secondary none" ANCHOR=sample_cand SKIP=0.6 SPAN=12000 bash scripts/tp1_trace.sh || exit $?
python scripts/step_breakdown.py gpurun_out/tp1_window.csv > gpurun_out/r4w/tp8sim_window.summary.txt
rm -f gpurun_out/tp1_window.csv
