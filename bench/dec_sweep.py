"""Decode-GEMM plan sweep at one M (default 64) for a model's projections: every gemm_mid tile x ring depth x
K split, weights rotated over > 600 MB (HBM-streamed, as in a decode step), graph-replay timing. Split plans of
the slab-consuming projections (qkv -> rope_cache, o / down -> add_norm at TP=1) are timed as partial outputs
and listed with the slab bytes the consumer must read; the others as in-launch combines (hint bit 256).

usage: python bench/dec_sweep.py [--model gpt2xl] [--m 64] [--top 8]
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"gpt2xl": {"qkv": (4800, 1600, "none", True), "o": (1600, 1600, "none", True),
                     "up": (6400, 1600, "gelu_tanh", False), "down": (1600, 6400, "none", True)}}
MID_BN = {7: 48, 14: 32, 15: 96, 11: 128, 13: 192, 10: 256}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2xl")
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--only-dec", action="store_true", help="only the K-split-wave decode kernel (gemm_dec.hip)")
    args = ap.parse_args()
    from llmss_amd.ops import autotune as A
    from llmss_amd.ops import hip as H

    dev = torch.device("cuda", 0)
    M = args.m
    for name, (N, K, act, partial) in SHAPES[args.model].items():
        if args.shapes and name not in args.shapes.split(","):
            continue
        ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
        base = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = [base.clone() for _ in range(ncopy)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        nk = -(-K // 64)
        res = []

        ref = x.float() @ ws[0].float().t()
        if act == "gelu_tanh":
            ref = torch.nn.functional.gelu(ref, approximate="tanh")

        def run(nt, s, part):
            def f(i):
                return H.linear(x, ws[i % ncopy], None, act, False, None, out=None if part else y, nt_hint=nt,
                                split_hint=s, partial_ok=part)
            r = f(0)
            torch.cuda.synchronize()
            slabs = r.S if isinstance(r, H.PartialSum) else 0
            got = r.buf[:slabs * M * N].view(slabs, M, N).sum(0) if slabs else r.float()
            err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
            if not err < 2e-2:
                raise SystemExit(f"{name} plan {hex(nt)} s{s}: max rel err {err:.3g}")
            return A._time(f, 16), slabs

        cands = []
        for code in (1, 2, 3, 4, 5):  # gemm_dec: hint bit 1024 of the tile bits
            for d in (0, 16, 32):
                for s in (1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 25):
                    if s > nk or -(-N // (16 * (1, 2, 3, 4, 6)[code - 1])) * s > 2048:
                        continue
                    if partial or s == 1:
                        cands.append(((code | d | 1024) << 8, s, partial and s > 1))
                    if 1 < s <= 4:  # split-K combined in the launch: finished output
                        cands.append(((code | d | 1024 | 256) << 8, s, False))
        for t, bn in ({} if args.only_dec else MID_BN).items():
            for d in (32, 48):
                for s in sorted({1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 13, 16, 20, 25}):
                    if s > 1 and nk // s < 1:
                        continue
                    tiles = -(-N // bn)
                    if tiles * s > 1024:
                        continue
                    if partial or s == 1:
                        cands.append(((t | d) << 8, s, partial))
                    if s > 1:
                        cands.append(((t | d | 256) << 8, s, False))
        for t, d in (() if args.only_dec else ((3, 32), (3, 48), (2, 32))):
            for s in (1, 2, 4, 5, 8):
                cands.append(((t | d) << 8, s, partial and s > 1))
        for nt, s, part in cands:
            try:
                us, slabs = run(nt, s, part)
            except (RuntimeError, ValueError) as e:  # noqa: PERF203
                if not res and not getattr(run, "told", False):
                    print(f"# {name} {hex(nt)} s{s}: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
                    run.told = True
                continue
            res.append({"nt": hex(nt), "s": s, "us": round(us, 2), "slabs": slabs,
                        "slab_MB": round(slabs * M * N * 4 / 1e6, 2)})
        res.sort(key=lambda r: r["us"])
        print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "MB": round(N * K * 2 / 1e6, 1),
                          "best": res[:args.top]}), flush=True)
        del ws


if __name__ == "__main__":
    main()
