"""Compact GEMM candidate probe: for each (shape, M) print hipBLASLt, the static plan, the autotuner's
candidate list (ops/autotune.py) ranked, and the best per kernel family - times per call measured
inside a HIP graph with weights rotated over > 2x the Infinity Cache (HBM-streamed, like decode).

usage: python bench/gemm_probe.py --shapes llama7b_tp8 --m 128,256,512 [--top 6] [--extra 0x1500:8,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import SHAPES, timeit  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402
from llmss_amd.ops.autotune import candidates  # noqa: E402


def family(nt: int) -> str:
    if nt == 0:
        return "static"
    if nt & 0xff:
        return f"stream_v{(nt >> 4) & 15}"
    t = nt >> 8
    if t & 128:
        return f"streamk_t{t & 15}"
    return {1: "128x128", 2: "64x128", 3: "64x64", 4: "big256", 5: "256x128w8", 6: "256x64w8"}.get(t & 15, f"t{t & 15}") \
        + f"_d{(t >> 4) & 3}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama7b_tp8")
    ap.add_argument("--m", default="128,256,512")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--extra", default="", help="extra nt:split pairs (hex nt ok)")
    ap.add_argument("--out", default="")
    ap.add_argument("--stream", action="store_true", help="add the weight-streaming kernels for any M <= 128")
    a = ap.parse_args()
    dev = torch.device("cuda")
    extra = [(int(p.split(":")[0], 0), int(p.split(":")[1])) for p in a.extra.split(",") if p]
    rows = []
    for sname in a.shapes.split(","):
        for name, N, K in SHAPES[sname]:
            glu = name == "gate_up"
            ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
            ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
            for M in [int(m) for m in a.m.split(",")]:
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                y = torch.empty(M, N // 2 if glu else N, device=dev, dtype=torch.bfloat16)
                yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                hb = timeit(lambda i: torch.matmul(x, ws[i % ncopy].t(), out=yb))
                res = []
                cands = candidates(M, N, K, glu, False)
                if a.stream and 32 < M <= 128:
                    cands += [(nt + 16 * v, s) for v in (1, 2) for nt in (1, 2) for s in (1, 2, 4, 8)]
                for nt, sp in [(0, 0)] + cands + extra:
                    try:
                        t = timeit(lambda i: H.linear(x, ws[i % ncopy], None, glu=glu, out=y, nt_hint=nt,
                                                      split_hint=sp), iters=30)
                    except (ValueError, RuntimeError):
                        continue
                    res.append((t, nt, sp))
                static = res[0][0]
                res.sort()
                fam = {}
                for t, nt, sp in res:
                    fam.setdefault(family(nt), (round(t, 2), hex(nt), sp))
                row = {"shape": sname, "layer": name, "M": M, "N": N, "K": K, "glu": glu,
                       "hipblaslt_us": round(hb, 2), "static_us": round(static, 2),
                       "best_TBps": round(N * K * 2 / res[0][0] / 1e6, 2), "hipblaslt_TBps": round(N * K * 2 / hb / 1e6, 2),
                       "top": [(round(t, 2), hex(nt), sp) for t, nt, sp in res[:a.top]], "by_family": fam}
                print(json.dumps(row), flush=True)
                rows.append(row)
            del ws
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
