"""Total / count / mean device time per kernel name in a rocprofv3 kernel-trace CSV (top N by total).

usage: python scripts/kernel_totals.py run_kernel_trace.csv [N] [--last-s S | --bench-log bench.log]
  --last-s S        only kernels that start in the last S seconds of the trace (the timed steps of a bench run)
  --bench-log LOG   S = the elapsed seconds of the last "[bench] step k: ... X s elapsed" line of bench.py's log
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("n", nargs="?", type=int, default=30)
    ap.add_argument("--last-s", type=float, default=0.0)
    ap.add_argument("--bench-log", default="")
    a = ap.parse_args()
    last = a.last_s
    if a.bench_log:
        for line in open(a.bench_log):
            m = re.search(r"\[bench\] step \d+: .* ([0-9.]+)s elapsed", line)
            if m:
                last = float(m.group(1))
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(a.csv))]
    if last > 0 and rows:
        t_end = max(e for _, e, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - last * 1e9]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for s, e, name in rows:
        x = agg[name[:70]]
        x[0] += (e - s) / 1e3
        x[1] += 1
    total = sum(t for t, _ in agg.values())
    print(f"window {last:.3f} s: {len(rows)} kernels, {total / 1e3:.1f} ms device time")
    for name, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.n]:
        print(f"{t:10.1f} us {c:6d} calls {t / c:8.2f} us/call {100 * t / total:5.1f}%  {name}")


if __name__ == "__main__":
    main()
