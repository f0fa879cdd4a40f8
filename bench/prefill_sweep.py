"""Prompt-batch GEMM sweep: every large-M plan on a model's projection shapes at M rows (default 8192: the
bench's 64 x 128-token prefill), timed as the autotuner times (HIP graph of calls, weights rotated past the
caches). One line per (shape, plan): us and TF/s.

usage: python bench/prefill_sweep.py [--model gpt2-xl] [--M 8192]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = {  # name: (N, K, glu, act)
    "gpt2-xl": {"qkv": (4800, 1600, False, "none"), "o": (1600, 1600, False, "none"),
                "up": (6400, 1600, False, "gelu_tanh"), "down": (1600, 6400, False, "none")},
    "llama2-7b": {"qkv": (12288, 4096, False, "none"), "o": (4096, 4096, False, "none"),
                  "up": (22016, 4096, True, "none"), "down": (4096, 11008, False, "none")},
}
PLANS = [  # (label, nt_hint, split)
    ("pp256x256", 4 << 8, 1),
    ("t256x128", (5 | 16) << 8, 1), ("t256x64", (6 | 16) << 8, 1), ("t128x128", 1 << 8, 1),
    ("t128x128d3", (1 | 16) << 8, 1), ("sk128x128g1", (1 | 128) << 8, 1), ("sk128x128g2", (1 | 128) << 8, 2),
    ("mid256x128", (9 | 16) << 8, 1), ("mid128x128", (8 | 16) << 8, 1), ("mid128x256", (12 | 16) << 8, 1),
    ("mid128x128ilv", (8 | 16 | 512) << 8, 1), ("mid128x128ilv4", (8 | 32 | 512) << 8, 1),
    ("mid256x128ilv", (9 | 16 | 512) << 8, 1), ("mid128x256ilv", (12 | 16 | 512) << 8, 1),
    ("mid64x256ilv", (10 | 16 | 512) << 8, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl", choices=sorted(SHAPES))
    ap.add_argument("--M", type=int, default=8192)
    a = ap.parse_args()
    from llmss_amd.ops import hip as H
    from llmss_amd.ops.autotune import _time

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    M = a.M
    for name, (N, K, glu, act) in SHAPES[a.model].items():
        x = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        base = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        ncopy = max(2, min(16, (600 << 20) // (N * K * 2)))
        ws = [base.clone() for _ in range(ncopy)]
        y = torch.empty(M, N // 2 if glu else N, dtype=torch.bfloat16, device=dev)
        ref = H.linear(x, ws[0], None, act, glu, out=torch.empty_like(y), nt_hint=4 << 8, split_hint=1)
        flops = 2.0 * M * N * K
        for label, nt, s in PLANS:
            try:
                out = H.linear(x, ws[0], None, act, glu, out=y, nt_hint=nt, split_hint=s)
                torch.cuda.synchronize()
                err = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
                us = _time(lambda i: H.linear(x, ws[i % ncopy], None, act, glu, out=y, nt_hint=nt, split_hint=s), 8)
            except (RuntimeError, ValueError) as e:
                print(f"{a.model} {name:5s} M={M} N={N} K={K} {label:15s} rejected: {str(e)[:80]}", flush=True)
                continue
            print(f"{a.model} {name:5s} M={M} N={N} K={K} {label:15s} {us:9.1f} us {flops / us * 1e-6:7.0f} TF/s "
                  f"maxrel {err:.1e}", flush=True)
        del ws


if __name__ == "__main__":
    main()
