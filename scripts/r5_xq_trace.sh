# round 5: kernel trace of bench/xq_probe.py (cross-stream dependency patterns, graph and eager)
set -u
mkdir -p gpurun_out/xq
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/xq/tr -o run --output-format csv -- python3 bench/xq_probe.py --us 20 --side-us 10 --n 8 > gpurun_out/xq/trace_run.log 2>&1 || { tail -20 gpurun_out/xq/trace_run.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/xq/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
with open("gpurun_out/xq/trace_compact.csv", "w") as o:
    o.write("queue,start_us,end_us,dur_us,name\n")
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        o.write(f"{r['Queue_Id']},{(s - t0) / 1e3:.2f},{(e - t0) / 1e3:.2f},{(e - s) / 1e3:.2f},{r['Kernel_Name'][:40]}\n")
PY
rm -rf gpurun_out/xq/tr
wc -l gpurun_out/xq/trace_compact.csv
