"""Table of per-dispatch PMC means for scripts/pmc_gemm_cfgs.sh output (kernels matching --match).
usage: python scripts/pmc_table.py OUTDIR [--match gemm_tiled]"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "gemm"
    cfgs = dict(l.strip().split(": ", 1) for l in open(os.path.join(d, "configs.txt")))
    rows = {}
    for c in sorted(cfgs):
        agg = collections.defaultdict(list)
        durs = []
        for run in glob.glob(os.path.join(d, f"{c}_p*")):
            for f in glob.glob(os.path.join(run, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if re.search(match, r["Kernel_Name"]):
                        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            for f in glob.glob(os.path.join(run, "**", "*kernel_trace.csv"), recursive=True):
                durs += [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f))
                         if re.search(match, r["Kernel_Name"])]
        row = {k: sum(v) / len(v) for k, v in agg.items()}
        if durs:
            durs.sort()
            row["median_us"] = durs[len(durs) // 2] / 1e3
        wc = row.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in row:
                    row[k + "_pct"] = round(100 * row[k] / wc, 1)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and "GRBM_GUI_ACTIVE" in row:
            # MFMA busy per SIMD relative to elapsed GPU cycles (1024 SIMDs; GRBM summed over 8 XCDs)
            row["mfma_util_pct"] = round(100 * row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] / 8 * 1024), 1)
        if "FETCH_SIZE" in row:
            row["fetch_MB_x2"] = round(row["FETCH_SIZE"] * 2 / 1024, 1)  # gfx950 FETCH_SIZE reads half of wide streams
        rows[c] = {"cfg": cfgs[c], **{k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}}
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
