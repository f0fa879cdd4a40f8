# GPU clock / power while the headline bench decodes (is the in-step slowdown a clock effect?)
set -u
mkdir -p gpurun_out/r4k
( for i in $(seq 1 40); do date +%s.%N; rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|Temperature \(Sensor (junction|memory)" ; sleep 1; done ) > gpurun_out/r4k/clocks.log 2>&1 &
SMI=$!
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --secondary none > gpurun_out/r4k/bench.log 2>&1
rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
exit $rc
