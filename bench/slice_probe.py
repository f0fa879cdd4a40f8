"""Weight-slice decode GEMM (csrc/gemm_slice.hip) against the autotuner's best other plan, per shape.

Weights rotate over > 600 MB of copies (HBM-cold, as in a decode step); each row prints the per-call time
of every slice configuration (nt, split) next to the best tuned plan of the remaining candidates.

usage: python bench/slice_probe.py [--shapes gpt2xl,llama7b] [--m 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402

SHAPES = {
    "gpt2xl": [("qkv", 4800, 1600), ("o", 1600, 1600), ("fc", 6400, 1600), ("proj", 1600, 6400)],
    "llama7b": [("qkv", 12288, 4096), ("o", 4096, 4096), ("down", 4096, 11008)],
    "llama7b_tp2": [("qkv", 6144, 4096), ("o", 4096, 2048), ("down", 4096, 5504)],
}


def time_plan(M, N, K, nt, split, dev, partial):
    """Per-call us of one (nt_hint, split) plan, HBM-cold weights, plus the consumer's slab reads (as the
    autotuner charges them)."""
    from llmss_amd.ops import hip as H

    ncopy = max(2, min(64, -(-(600 << 20) // (N * K * 2))))
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    base = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    ws = [base.clone() for _ in range(ncopy)]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)

    def f(i):
        return H.linear(x, ws[i % ncopy], None, out=None if partial else y, nt_hint=nt, split_hint=split,
                        partial_ok=partial)
    r = f(0)
    slabs = r.S if isinstance(r, H.PartialSum) else 0
    torch.cuda.synchronize()
    t = A._time(f, 16)
    return t + (slabs * M * N * 4 / A._SLAB_READ_BPS * 1e6 if slabs else 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="gpt2xl,llama7b")
    ap.add_argument("--m", default="64")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for sname in a.shapes.split(","):
        for M in (int(m) for m in a.m.split(",")):
            for lname, N, K in SHAPES[sname]:
                partial = lname in ("qkv", "o", "proj", "down")
                shp = A.GemmShape(N, K, partial=partial)
                cands = A.candidates(M, N, K, False, False)
                others = [c for c in cands if (c[0] & 0xff) >> 4 != 3]
                slices = [c for c in cands if (c[0] & 0xff) >> 4 == 3]
                nt, s, t_best, t_static = A.tune_shape(M, shp, dev, cands=others)
                row = {"shape": sname, "layer": lname, "M": M, "N": N, "K": K,
                       "best_other": [hex(nt), s, round(t_best, 2)], "static": round(t_static, 2), "slice_us": {}}
                for c in slices:
                    try:
                        row["slice_us"][f"nt{c[0] & 15}s{c[1]}"] = round(time_plan(M, N, K, c[0], c[1], dev, partial), 2)
                    except (RuntimeError, ValueError) as e:
                        row["slice_us"][f"nt{c[0] & 15}s{c[1]}"] = str(e)[:40]
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
