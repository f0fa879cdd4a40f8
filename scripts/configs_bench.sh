# One bench line per BASELINE.json config that fits one MI355X (+ batch sweep of the headline model).
mkdir -p gpurun_out/configs
run() { name=$1; shift; echo "=== $name"; timeout -k 10 ${TO:-300} python bench.py "$@" > gpurun_out/configs/$name.log 2>&1; rc=$?; tail -1 gpurun_out/configs/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
run gpt2xl_tp1 --model gpt2-xl
run llama7b_tp1_b128 --batch-per-gpu 128
run llama7b_tp1_b256 --batch-per-gpu 256
run llama13b_tp1 --model llama2-13b
TO=500 run llama70b_fp8_tp1 --model llama2-70b --fp8 --steps 2
TO=500 run llama70b_fp8_tp8sim --model llama2-70b --fp8 --simulate-tp 8 --steps 2
