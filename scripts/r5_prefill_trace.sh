# round 5: kernel trace of the headline bench to take the prompt-batch (prefill) step apart
set -u
mkdir -p gpurun_out/r5pt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5pt/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --secondary none > gpurun_out/r5pt/bench.log 2>&1 || { tail -20 gpurun_out/r5pt/bench.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r5pt/tr/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pp = [i for i, r in enumerate(rows) if "gemm_pp_kernel" in r["Kernel_Name"]]
# clusters of pp kernels separated by > 50 ms
cl, cur = [], [pp[0]]
for a, b in zip(pp, pp[1:]):
    if int(rows[b]["Start_Timestamp"]) - int(rows[a]["End_Timestamp"]) > 50e6:
        cl.append(cur); cur = []
    cur.append(b)
cl.append(cur)
last = cl[-1]
i0, i1 = last[0], last[-1]
# extend to the embed before the first pp and to the first sample after the last pp
while i0 > 0 and "embed" not in rows[i0]["Kernel_Name"]:
    i0 -= 1
while i1 < len(rows) - 1 and "sample" not in rows[i1]["Kernel_Name"]:
    i1 += 1
t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[i1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[i0:i1 + 1]:
    k = r["Kernel_Name"][:70]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
with open("gpurun_out/r5pt/prefill_step.summary.txt", "w") as f:
    f.write(f"prefill step window {(t1 - t0) / 1e3:.1f} us, {i1 - i0 + 1} kernels, busy {busy:.1f} us, pp clusters {len(cl)}\n")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        f.write(f"  {k:70s} {us:9.1f} us {n:5d} calls {us / n:8.2f} us/call\n")
print(open("gpurun_out/r5pt/prefill_step.summary.txt").read())
PY
rm -f gpurun_out/r5pt/tr/*kernel_trace.csv
