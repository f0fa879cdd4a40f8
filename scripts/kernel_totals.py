"""Total / count / mean device time per kernel name in a rocprofv3 kernel-trace CSV (top N by total).

usage: python scripts/kernel_totals.py run_kernel_trace.csv [N]
"""
import collections
import csv
import sys


def main(path, n=30):
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg[r["Kernel_Name"][:70]]
        a[0] += d
        a[1] += 1
    for name, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:n]:
        print(f"{t:10.1f} us {c:6d} calls {t / c:8.2f} us/call  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
