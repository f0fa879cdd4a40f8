#!/bin/bash
# GPU box check: kernel numerics -> engine tests -> smoke -> short bench -> rocprof stats.
# Every GPU step has its own time limit; the script stops at the first crash/timeout
# (exit status other than 0 or 1 = pytest "tests failed").
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
ok() { [ "$1" -eq 0 ] || { [ "$1" -eq 1 ] && [ -n "${KEEP_GOING:-}" ]; }; }
STAGES=${STAGES:-"kernels engine smoke bench"}
for s in $STAGES; do
  case $s in
    kernels) step kernels 900 python -m pytest tests/test_kernels_gpu.py -q -rf --timeout 300; rc=$? ;;
    engine) step engine 900 python -m pytest tests/test_engine_gpu.py -q -rf --timeout 300; rc=$? ;;
    gputests) step gputests 1200 python -m pytest tests -m gpu -q -rf --timeout 600; rc=$? ;;
    gemm) step gemm 380 python bench/gemm_bench.py ${GEMM_ARGS:-}; rc=$? ;;
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"; rc=$? ;;
    bench) step bench 380 python bench.py ${BENCH_ARGS:-}; rc=$? ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null;
          step prof 380 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:-}; rc=$?
          rm -f gpurun_out/prof/*kernel_trace.csv ;;
    prof8) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null;
          step prof8 380 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --simulate-tp 8; rc=$?
          rm -f gpurun_out/prof8/*kernel_trace.csv ;;
    *) echo "unknown stage $s"; rc=2 ;;
  esac
  ok $rc || { echo "stopping after $s (rc=$rc)"; exit $rc; }
done
