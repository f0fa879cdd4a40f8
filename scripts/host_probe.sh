# host-side cost of the TP=8 shard's decode loop (batch 512): engine host phase timers + cProfile of bench.py
mkdir -p gpurun_out/host
LLMSS_HOST_PROFILE=1 timeout -k 10 600 python -m cProfile -o gpurun_out/host/bench.prof bench.py --simulate-tp 8 --steps 1 --warmup 1 --secondary none > gpurun_out/host/bench.log 2>&1 || exit $?
python - <<'PY' > gpurun_out/host/profile_top.txt
import pstats
p = pstats.Stats("gpurun_out/host/bench.prof")
p.sort_stats("tottime").print_stats(40)
PY
rm -f gpurun_out/host/bench.prof
grep -o '"engine_stats": {[^}]*}' gpurun_out/host/bench.log
