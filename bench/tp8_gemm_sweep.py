"""Sweep every autotuner candidate on the per-rank decode GEMMs of Llama-2-7B at TP=8 (M=512 rows: 64
requests per GPU x 8 ranks) and print the fastest plans per shape and per tile family, in-graph and with
HBM-streamed weights like ops/autotune.py tune_shape.

usage: python bench/tp8_gemm_sweep.py [--m 512] [--top 8] [--shapes qkv,o,up,down] [--extra HINT,SPLIT ...]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as AT  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402

# name -> (N, K, glu, consumer sums split-K slabs itself); Llama-2-7B / TP=8: 4096 hidden, 11008 MLP
SHAPES = {"qkv": (1536, 4096, False, True), "o": (4096, 512, False, False), "up": (2752, 4096, True, False),
          "down": (4096, 1376, False, False)}
# TP=1 (--tp1): o / down partials are summed by the next add_norm
SHAPES_TP1 = {"qkv": (12288, 4096, False, True), "o": (4096, 4096, False, True), "up": (22016, 4096, True, False),
              "down": (4096, 11008, False, True)}


def family(nt: int) -> str:
    t = (nt >> 8) & 15
    flags = (nt >> 8) & ~63
    tag = {1: "128x128", 2: "64x128", 3: "64x64", 4: "big256", 5: "256x128t", 6: "256x64t", 7: "mid64x48",
           8: "mid128x128", 9: "mid256x128", 10: "mid64x256", 11: "mid64x128", 12: "mid128x256", 13: "mid64x192",
           14: "mid64x32", 15: "mid64x96"}.get(t, f"t{t}")
    if flags & 128:
        tag += "+sk"
    if flags & 256:
        tag += "+comb"
    if flags & 512:
        tag += "+ilv"
    return tag


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--shapes", default="qkv,o,up,down")
    ap.add_argument("--extra", nargs="*", default=[], help="additional HINT,SPLIT plans (hex ok)")
    ap.add_argument("--tp1", action="store_true", help="Llama-2-7B TP=1 shapes instead of the TP=8 shard")
    ap.add_argument("--deep", action="store_true", help="add deeper LDS rings (depth code 48) of the gemm_mid tiles")
    ap.add_argument("--warm", action="store_true", help="one weight copy (cache-resident) instead of HBM-streamed")
    a = ap.parse_args()
    dev = torch.device("cuda")
    M = a.m
    total_best = 0.0
    for name in a.shapes.split(","):
        N, K, glu, partial = (SHAPES_TP1 if a.tp1 else SHAPES)[name]
        ncopy = 1 if a.warm else max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
        base = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = [base.clone() for _ in range(ncopy)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        y = torch.empty(M, N // 2 if glu else N, dtype=torch.bfloat16, device=dev)
        cands = [(0, 0)] + AT.candidates(M, N, K, glu, False)
        cands += [tuple(int(v, 0) for v in e.split(",")) for e in a.extra]
        if a.deep:
            nk = -(-K // 64)
            cands += [(((t | 48) << 8), sp) for t in (11, 13, 15, 10, 8) for sp in (1, 2, 3, 4, 5, 6, 8)
                      if sp == 1 or nk // sp >= 2]
        res = []
        for nt, s in cands:
            for fin in ((True, False) if partial else (True,)):
                def f(i, nt=nt, s=s, fin=fin):
                    return H.linear(x, ws[i % ncopy], None, glu=glu, out=y if fin else None, nt_hint=nt,
                                    split_hint=s, partial_ok=not fin)
                try:
                    r = f(0)
                    slabs = r.S if isinstance(r, H.PartialSum) else 0
                    f(1)
                    torch.cuda.synchronize()
                    t = AT._time(f, 16)
                except (ValueError, RuntimeError):
                    continue
                # a consumer that sums the slabs pays their reads (ops/autotune.py _SLAB_READ_BPS)
                t_eff = t + (slabs * M * N * 4 / AT._SLAB_READ_BPS * 1e6 if slabs else 0.0)
                res.append((t_eff, t, nt, s, fin, slabs))
        res.sort()
        flop = 2 * M * N * K
        print(f"== {name}{' (warm)' if a.warm else ''}: M={M} N={N} K={K} glu={glu}  ({flop / 1e9:.1f} GFLOP, {N * K * 2 / 1e6:.1f} MB weights)")
        for t_eff, t, nt, s, fin, slabs in res[:a.top]:
            print(f"  {t_eff:7.2f} us (kernel {t:6.2f}, slabs {slabs})  {nt:#07x}/s{s:<2} {family(nt):14s} "
                  f"{'final' if fin else 'partial'}  {flop / t_eff / 1e6:6.0f} TF/s")
        best = {}
        for r in res:
            fam = family(r[2])
            if fam not in best:
                best[fam] = r
        print("  best per family: " + ", ".join(f"{k} {v[0]:.1f}" for k, v in sorted(best.items(), key=lambda kv: kv[1][0])))
        total_best += res[0][0]
        del ws
        torch.cuda.empty_cache()
    print(f"sum of best: {total_best:.1f} us per layer", flush=True)


if __name__ == "__main__":
    main()
