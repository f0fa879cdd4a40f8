#!/bin/bash
# Counter collection for one decode GEMM shape (own run: --pmc with kernel-trace only).
set -u
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || true
i=0
for PMC in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC -d gpurun_out/pmc/run$i -o pmc --output-format csv -- \
    python3 bench/gemm_one.py ${GEMM_ONE_ARGS:-} > gpurun_out/pmc/run$i.log 2>&1 || echo "pmc run $i failed rc=$?"
done
