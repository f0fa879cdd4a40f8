"""Compact view of bench/gemm_bench.py --sweep output: hipBLASLt, default plan, overall best and the
best configuration of each tile family (tiled hint = nt >> 8: tile = & 15, stream-K = & 128)."""
import json
import sys

FAM = {1: "128x128", 2: "64x128", 3: "64x64", 4: "256x256", 5: "256x128w8", 6: "256x64w8"}
for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        fam = {}
        for k, v in d.items():
            if not (k.startswith("nt") and k.endswith("_us")):
                continue
            nt, sp = k[2:-3].split("_s")
            t = int(nt) >> 8
            name = ("sk-" if t & 128 else "") + FAM.get(t & 15, "stream") if t else "stream"
            if name not in fam or v < fam[name][0]:
                fam[name] = (v, f"{int(nt):#x}/s{sp}")
        fams = " ".join(f"{n}={v[0]:.1f}({v[1]})" for n, v in sorted(fam.items(), key=lambda x: x[1][0])[:4])
        print(f"{d['shape']:12s} {d['layer']:8s} M={d['M']:4d} blas={d.get('hipblaslt_us')} ours={d.get('ours_us')} | {fams}")
