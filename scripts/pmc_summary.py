"""Summarise rocprofv3 PMC runs written by scripts/pmc_gemm.sh: mean counter value per dispatch of
kernels whose name contains --match, plus the median kernel duration.

usage: python scripts/pmc_summary.py gpurun_out/pmc_* [--match gemm]
"""
import collections
import csv
import glob
import os
import sys


def summarise(d, match):
    out = {}
    for run in sorted(glob.glob(os.path.join(d, "run*/"))):
        for f in glob.glob(os.path.join(run, "*counter_collection.csv")):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                if match in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            out.update({k: round(sum(v) / len(v)) for k, v in agg.items()})
        for f in glob.glob(os.path.join(run, "*kernel_trace.csv")):
            dur = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f))
                         if match in r["Kernel_Name"])
            if dur:
                out.setdefault("median_us", dur[len(dur) // 2] / 1e3)
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "gemm"
    args = [a for a in args if a != match]
    for d in args:
        print(os.path.basename(d.rstrip("/")), summarise(d, match))
