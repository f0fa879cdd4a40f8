mkdir -p gpurun_out/dual
MODEL=gpt2-xl timeout -k 10 300 python bench/dual_stream_probe.py > gpurun_out/dual/gpt2xl.log 2>&1 &&
MODEL=llama2-7b timeout -k 10 300 python bench/dual_stream_probe.py > gpurun_out/dual/llama7b.log 2>&1
rc=$?; tail -n 2 gpurun_out/dual/*.log; exit $rc
