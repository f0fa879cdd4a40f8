"""Every autotuner candidate of one decode shape, timed as the autotuner times it (HIP graph, HBM-cold weights):
prints the fastest plans with their weight streaming rate. Raw slab time (no slab-read charge) is shown too.

usage: python bench/plan_dump.py M N K [--glu] [--top 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--glu", action="store_true")
    ap.add_argument("--partial", action="store_true", help="consumer sums split-K slabs (qkv / o / down at TP=1)")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    shp = A.GemmShape(a.N, a.K, a.glu, False, a.partial, "none")
    ncopy = max(2, min(64, -(-(600 << 20) // (a.N * a.K * 2))))
    x = (torch.randn(a.M, a.K, device=dev) * 0.5).to(torch.bfloat16)
    base = (torch.randn(a.N, a.K, device=dev) * a.K ** -0.5).to(torch.bfloat16)
    ws = [base.clone() for _ in range(ncopy)]
    y = torch.empty(a.M, a.N // 2 if a.glu else a.N, dtype=torch.bfloat16, device=dev)
    rows = []
    for nt, s in [(0, 0)] + A.candidates(a.M, a.N, a.K, a.glu, False):
        def f(i, nt=nt, s=s):
            return H.linear(x, ws[i % ncopy], None, "none", a.glu, None, out=None if shp.partial else y,
                            nt_hint=nt, split_hint=s, partial_ok=shp.partial)
        try:
            r = f(0)
            slabs = r.S if isinstance(r, H.PartialSum) else 0
            torch.cuda.synchronize(dev)
            t = A._time(f, 16)
        except (ValueError, RuntimeError):
            continue
        rows.append((t, nt, s, slabs))
    rows.sort()
    wb = a.N * a.K * 2
    print(f"M={a.M} N={a.N} K={a.K} glu={a.glu} partial={a.partial}: {len(rows)} plans")
    for t, nt, s, slabs in rows[:a.top]:
        print(f"  0x{nt:x}/s{s}  {t:6.1f} us  {wb / t / 1e6:5.2f} TB/s  slabs {slabs}")


if __name__ == "__main__":
    main()
