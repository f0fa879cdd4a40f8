# PMC passes of the prefill GEMM prototypes (bench/proto/pp_gemm.hip) on the Llama qkv shape at M = 8192.
# Each pass is its own run (--pmc with --kernel-trace only); VARS picks the arms.
set -u
mkdir -p gpurun_out/r5p
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
VARS=${VARS:-2,4}
A="--m 8192 --shapes ${SHAPE:-qkv} --vars $VARS --rounds 1 --iters 10 --no-big --no-lib"
timeout -k 10 -s KILL 90 rocprofv3 -L > gpurun_out/r5p/counters.txt 2>&1 || true
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r5p/p1 -o pmc --output-format csv -- python3 bench/pp_probe.py $A > gpurun_out/r5p/p1.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC -d gpurun_out/r5p/p2 -o pmc --output-format csv -- python3 bench/pp_probe.py $A > gpurun_out/r5p/p2.log 2>&1 || exit 1
rm -f gpurun_out/r5p/*/pmc_kernel_trace.csv
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/r5p/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gemm" not in k:
                continue
            agg[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(p, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
