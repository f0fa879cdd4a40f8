"""Time GEMM plans with and without the in-launch split-K combine (hint bit 256) on decode shapes.

usage: python bench/combine_probe.py [--shapes gpt2|tp8|tp1|all]
For each shape prints the static plan, the best slab plan (split-K partials + reduce launch, or no
split), the best combine plan and the best of each family's top candidates. Timing = autotune's:
calls captured in one HIP graph, weights rotating over > 600 MB of copies (HBM-cold).
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402

SHAPES = {
    # name: (M, N, K, act, glu)
    "gpt2": [("fc", 64, 6400, 1600, "gelu_tanh", False), ("o", 64, 1600, 1600, "none", False),
             ("proj", 64, 1600, 6400, "none", False), ("qkv", 64, 4800, 1600, "none", False)],
    "tp8": [("qkv", 512, 1536, 4096, "none", False), ("gate_up", 512, 2752, 4096, "none", True),
            ("o", 512, 4096, 512, "none", False), ("down", 512, 4096, 1376, "none", False)],
    "tp1": [("qkv", 64, 12288, 4096, "none", False), ("gate_up", 64, 22016, 4096, "none", True),
            ("o", 64, 4096, 4096, "none", False), ("down", 64, 4096, 11008, "none", False)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--stream", action="store_true", help="also time the weight-streaming kernels (nt + 16 * variant)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    H.reserve_workspace(dev)
    groups = list(SHAPES) if a.shapes == "all" else a.shapes.split(",")
    for grp in groups:
        for name, M, N, K, act, glu in SHAPES[grp]:
            ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            base = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
            ws = [base.clone() for _ in range(ncopy)]
            y = torch.empty(M, N // 2 if glu else N, dtype=torch.bfloat16, device=dev)

            def cost(nt, s):
                def f(i):
                    H.linear(x, ws[i % ncopy], None, act, glu, None, out=y, nt_hint=nt, split_hint=s)
                f(0)
                f(1)
                torch.cuda.synchronize()
                return A._time(f, a.iters)

            res = {"slab": [], "comb": [], "stream": []}
            cands = list(A.candidates(M, N, K, glu, False))
            if a.stream:
                cands += [(nt + 16 * v, s) for v in (1, 2) for nt in (1, 2) for s in (1, 2, 4, 8)]
            for nt, s in cands:
                try:
                    t = cost(nt, s)
                except (RuntimeError, ValueError):
                    continue
                res["stream" if nt & 0xff else ("comb" if (nt >> 8) & 256 else "slab")].append((t, nt, s))
            t0 = cost(0, 0)
            line = f"{grp:5s} {name:8s} M={M:4d} N={N:5d} K={K:5d} static {t0:6.1f}us"
            for k in ("slab", "comb", "stream"):
                top = sorted(res[k])[:3]
                line += f" | {k}: " + ", ".join(f"{t:.1f} ({nt:#x}/s{s})" for t, nt, s in top)
            print(line, flush=True)
            del ws


if __name__ == "__main__":
    main()
