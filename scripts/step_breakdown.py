"""Per-kernel time and inter-kernel gaps inside a window of a compact trace (scripts/trace_window.py
output): where one decode step's wall time goes."""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: float(r["start_us"]))
    tot = defaultdict(lambda: [0.0, 0])
    gaps = 0.0
    prev_end = None
    for r in rows:
        s, e = float(r["start_us"]), float(r["end_us"])
        k = r["name"]
        tot[k][0] += e - s
        tot[k][1] += 1
        if prev_end is not None and s > prev_end:
            gaps += s - prev_end
        prev_end = max(prev_end or 0, e)
    span = prev_end - float(rows[0]["start_us"])
    busy = sum(v[0] for v in tot.values())
    print(f"window {span:.1f} us, kernels {len(rows)}, busy {busy:.1f} us, gaps {gaps:.1f} us")
    for k, (t, n) in sorted(tot.items(), key=lambda x: -x[1][0]):
        print(f"  {k:50s} {t:9.1f} us {n:5d} calls {t / n:7.2f} us/call {100 * t / span:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1])
