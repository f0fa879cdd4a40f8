"""Per-stream busy time and cross-stream overlap inside a trace window (scripts/trace_window.py output): how much
of the comm stream's time ran beside compute, and the per-kernel table of each stream.

usage: python scripts/stream_overlap.py WINDOW.csv
"""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    tot = 0.0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path):
    rows = list(csv.DictReader(open(path)))
    key = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"  # kernel-trace alone leaves Stream_Id 0
    by = defaultdict(list)
    for r in rows:
        by[r[key]].append(r)
    t0 = min(float(r["start_us"]) for r in rows)
    t1 = max(float(r["end_us"]) for r in rows)
    print(f"window {t1 - t0:.1f} us, {len(rows)} kernels, streams {sorted(by)}")
    ivs = {k: union([(float(r["start_us"]), float(r["end_us"])) for r in v]) for k, v in by.items()}
    allu = union([x for v in ivs.values() for x in v])
    print(f"GPU busy (any stream) {length(allu):.1f} us = {100 * length(allu) / (t1 - t0):.1f} %")
    ks = sorted(by, key=lambda k: -length(ivs[k]))
    for k in ks:
        tot = defaultdict(lambda: [0.0, 0])
        for r in by[k]:
            tot[r["name"]][0] += float(r["dur_us"])
            tot[r["name"]][1] += 1
        print(f"stream {k}: busy {length(ivs[k]):.1f} us, {len(by[k])} kernels")
        for n, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:12]:
            print(f"    {n:50s} {t:9.1f} us {c:5d} calls {t / c:7.2f} us/call")
    if len(ks) > 1:
        main_s, others = ks[0], ks[1:]
        for o in others:
            ov = intersect(ivs[main_s], ivs[o])
            print(f"stream {o} beside stream {main_s}: {ov:.1f} us of its {length(ivs[o]):.1f} us overlapped")


if __name__ == "__main__":
    main(sys.argv[1])
