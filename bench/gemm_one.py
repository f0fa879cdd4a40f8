"""Run one GEMM configuration repeatedly (for rocprofv3 counter collection).

usage: python bench/gemm_one.py --m 64 --n 12288 --k 4096 [--hint 0x300 --split 4] [--iters 200]
Weights rotate over copies > 2x the Infinity Cache so every call streams from HBM.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--n", type=int, default=12288)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--hint", type=lambda v: int(v, 0), default=0)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--glu", action="store_true")
    ap.add_argument("--w8a8", default="", help="TILE,DEPTH: fp8 weights and per-token fp8 activations (W8A8)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    eb = 1 if a.w8a8 else 2  # weight bytes per element
    ncopy = max(2, int(600e6 // (a.n * a.k * eb)) + 1)
    ws = [(torch.randn(a.n, a.k, device=dev) * a.k ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
    scales = None
    if a.w8a8:
        q = [H.quant_fp8_rows(w) for w in ws]
        ws, scales = [t[0] for t in q], [t[1] for t in q]
        tile, depth = (int(v) for v in a.w8a8.split(","))
    x = torch.randn(a.m, a.k, device=dev).to(torch.bfloat16)
    y = torch.empty(a.m, a.n // 2 if a.glu else a.n, device=dev, dtype=torch.bfloat16)

    def call(i):
        if a.w8a8:
            H.linear_w8a8(x, ws[i % ncopy], scales[i % ncopy], None, glu=a.glu, out=y, tile=tile, depth=depth,
                          split=a.split)
        else:
            H.linear(x, ws[i % ncopy], None, glu=a.glu, out=y, nt_hint=a.hint, split_hint=a.split)

    for i in range(a.iters):
        call(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(a.iters):
        call(i)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / a.iters
    print(f"M={a.m} N={a.n} K={a.k} hint={a.hint:#x} w8a8={a.w8a8} split={a.split}: {us:.2f} us, "
          f"{a.n * a.k * eb / us / 1e6:.3f} TB/s weights")


if __name__ == "__main__":
    main()
