"""Where does a GPT-2-XL decode GEMM's time go: HBM streaming, or the kernel's own structure?

For each GPT-2-XL projection at M = 64 the autotuner's best plan is timed three ways (graph replay, no profiler):
  hbm   - weights rotated over > 600 MB, every call streams from HBM (the decode-step condition);
  mall  - one weight copy, re-read every call (resident in the 256 MiB Infinity Cache);
  pref  - rotated copies, but each GEMM is preceded by a read-everything kernel over the same weights
          (torch sum), reported as (pair - prefetch alone): the GEMM's time when its weights were just pulled
          into the Infinity Cache by the kernel before it.
usage: python bench/mall_probe.py [--m 64]
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"qkv": (4800, 1600), "o": (1600, 1600), "up": (6400, 1600), "down": (1600, 6400)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    args = ap.parse_args()
    from llmss_amd.ops import autotune as A
    from llmss_amd.ops import hip as H

    dev = torch.device("cuda", 0)
    M = args.m
    for name, (N, K) in SHAPES.items():
        act = "gelu_tanh" if name == "up" else "none"
        shp = A.GemmShape(N, K, False, False, False, act)
        nt, s, t_hbm, t_def = A.tune_shape(M, shp, dev)
        ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        sink = torch.empty(ncopy, N, dtype=torch.float32, device=dev)

        def gemm(i, c=None):
            H.linear(x, ws[(i % ncopy) if c is None else c], None, act, False, None, out=y, nt_hint=nt, split_hint=s)

        def pre(i):
            torch.sum(ws[i % ncopy], dim=1, dtype=torch.float32, out=sink[i % ncopy])

        def pair(i):
            pre(i)
            gemm(i)

        for f in (gemm, pre, pair):
            f(0)
        torch.cuda.synchronize()
        t_mall = A._time(lambda i: gemm(i, 0), 32)
        t_rot = A._time(gemm, 32)
        t_pre = A._time(pre, 32)
        t_pair = A._time(pair, 32)
        mb = N * K * 2 / 1e6
        rec = {"shape": name, "N": N, "K": K, "M": M, "plan": [hex(nt), s], "MB": round(mb, 1),
               "hbm_us": round(t_rot, 2), "tuned_us": round(t_hbm, 2), "static_us": round(t_def, 2),
               "mall_us": round(t_mall, 2), "prefetch_us": round(t_pre, 2), "pair_us": round(t_pair, 2),
               "after_prefetch_us": round(t_pair - t_pre, 2),
               "hbm_TBps": round(mb / t_rot, 2), "mall_TBps": round(mb / t_mall, 2)}
        print(json.dumps(rec), flush=True)
        del ws


if __name__ == "__main__":
    main()
