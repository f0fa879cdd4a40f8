"""Tuned HIP GEMMs (what the engine runs after autotuning) vs hipBLASLt (torch.matmul) on the layer
shapes of the benchmark models, at decode / mid-M batch sizes.

usage: python bench/gemm_vs_blaslt.py [--shapes llama7b,llama7b_tp8,gpt2xl] [--m 64,128,256,512]
One JSON line per (shape, layer, M): hipblaslt_us, static_us (planner), tuned_us + plan (autotuner
winner over its full candidate list), all with finished bf16 outputs (no slabs left to a consumer)
and weights rotating over > 600 MB of copies (HBM-cold), timed as HIP-graph replays. A summary
table follows on stderr.
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402

SHAPES = {
    "llama7b": [("qkv", 12288, 4096, False), ("o", 4096, 4096, False), ("gate_up", 22016, 4096, True),
                ("down", 4096, 11008, False)],
    "llama7b_tp8": [("qkv", 1536, 4096, False), ("o", 4096, 512, False), ("gate_up", 2752, 4096, True),
                    ("down", 4096, 1376, False)],
    "llama13b_tp8": [("qkv", 1920, 5120, False), ("o", 5120, 640, False), ("gate_up", 3456, 5120, True),
                     ("down", 5120, 1728, False)],
    "gpt2xl": [("qkv", 4800, 1600, False), ("o", 1600, 1600, False), ("fc", 6400, 1600, False),
               ("proj", 1600, 6400, False)],
}


def blaslt_us(M, N, K, glu, dev, iters=16):
    """torch.matmul (hipBLASLt) on the same HBM-cold weight rotation; SwiGLU layers pay only the
    matmul (the activation would be one more kernel for them)."""
    ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
    base = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    ws = [base.clone() for _ in range(ncopy)]
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)

    def f(i):
        torch.matmul(x, ws[i % ncopy].t(), out=y)
    f(0)
    torch.cuda.synchronize()
    t = A._time(f, iters)
    del ws
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama7b,llama7b_tp8,gpt2xl")
    ap.add_argument("--m", default="64,128,256,512")
    a = ap.parse_args()
    dev = torch.device("cuda")
    H.reserve_workspace(dev)
    rows = []
    for sname in a.shapes.split(","):
        for name, N, K, glu in SHAPES[sname]:
            for M in [int(v) for v in a.m.split(",")]:
                hb = blaslt_us(M, N, K, glu, dev)
                nt, s, t, t0 = A.tune_shape(M, A.GemmShape(N, K, glu), dev)
                r = {"shape": sname, "layer": name, "M": M, "N": N, "K": K, "glu": glu, "hipblaslt_us": round(hb, 2),
                     "static_us": round(t0, 2), "tuned_us": round(t, 2), "plan": [hex(nt), s],
                     "tuned_TBps": round(N * K * 2 / t / 1e6, 2), "tuned_TFLOPs": round(2 * M * N * K / t / 1e6, 1),
                     "vs_hipblaslt": round(hb / t, 3)}
                print(json.dumps(r), flush=True)
                rows.append(r)
                torch.cuda.empty_cache()
    print(f"{'shape':13s} {'layer':8s} {'M':>4s} {'hipBLASLt':>9s} {'ours':>7s} {'x':>6s}", file=sys.stderr)
    for r in rows:
        print(f"{r['shape']:13s} {r['layer']:8s} {r['M']:4d} {r['hipblaslt_us']:9.1f} {r['tuned_us']:7.1f} "
              f"{r['vs_hipblaslt']:6.2f}", file=sys.stderr)
    wins = sum(r["vs_hipblaslt"] >= 1.0 for r in rows)
    print(f"ours <= hipBLASLt on {wins}/{len(rows)} rows", file=sys.stderr)


if __name__ == "__main__":
    main()
