"""Cut a rocprofv3 kernel trace down to a time window: one compact CSV row per kernel
(short name, queue/stream ids, start/end us relative to the window) - for reading overlap and gaps.

usage: python scripts/trace_window.py TRACE.csv OUT.csv [--skip-frac 0.7] [--span-us 20000]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--skip-frac", type=float, default=0.7)
    ap.add_argument("--span-us", type=float, default=20000)
    ap.add_argument("--anchor", default="", help="start the window at the end of the middle occurrence of "
                                               "this kernel name (e.g. sample_v3: between two decode steps)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t_first, t_last = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    t0 = t_first + a.skip_frac * (t_last - t_first)
    if a.anchor:
        hits = [r for r in rows if a.anchor in r["Kernel_Name"]]
        if hits:
            t0 = int(hits[int(len(hits) * a.skip_frac)]["End_Timestamp"]) - 1000
    t1 = t0 + a.span_us * 1e3
    keys = [k for k in ("Queue_Id", "Stream_Id") if k in rows[0]]
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name"] + keys + ["start_us", "end_us", "dur_us"])
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < t0 or s > t1:
                continue
            nm = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
            w.writerow([nm] + [r[k] for k in keys] + [round((s - t0) / 1e3, 2), round((e - t0) / 1e3, 2),
                                                      round((e - s) / 1e3, 2)])


if __name__ == "__main__":
    main()
