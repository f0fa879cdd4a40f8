# round 5: HBM / L2 traffic of gemm_pp on the TP=8 qkv prompt-batch shape (M=65536, N=1536) vs the TP=1 one
# (M=8192, N=12288): same FLOPs, same K, same tile count, 20 % apart. One pass per counter group.
set -u
mkdir -p gpurun_out/r5pm
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for sh in "tp8_qkv 65536" "qkv 8192"; do
  set -- $sh
  A="--m $2 --shapes $1 --vars '' --rounds 1 --iters 3 --no-lib"
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r5pm/$1_f -o pmc --output-format csv -- python3 bench/pp_probe.py --m $2 --shapes $1 --vars "" --rounds 1 --iters 3 --no-lib > gpurun_out/r5pm/$1_f.log 2>&1 || exit 1
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r5pm/$1_h -o pmc --output-format csv -- python3 bench/pp_probe.py --m $2 --shapes $1 --vars "" --rounds 1 --iters 3 --no-lib > gpurun_out/r5pm/$1_h.log 2>&1 || exit 1
done
rm -f gpurun_out/r5pm/*/pmc_kernel_trace.csv
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r5pm/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gemm_pp" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
