"""Prompt-batch GEMM plans at large M: every in-tree kernel family a prefill projection can run on (ping-pong
256x256, 8-wave 256x128 / 256x64, 128x128 tiled and stream-K, gemm_mid 256x128 / 128x256 / 128x128 with and
without the interleaved ring), timed in a HIP graph per shape, with hipBLASLt (torch.matmul) as the yardstick.

usage: python bench/prefill_plan_probe.py [--m 65536,8192] [--shapes llama7b_tp8]
"""
import argparse
import json
import os
import sys

import torch
from typing import List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

from gemm_bench import SHAPES, timeit  # noqa: E402

from llmss_amd.ops import hip as H  # noqa: E402


def prefill_candidates(M: int, N: int, K: int, glu: bool) -> List[Tuple[int, int]]:
    """(nt_hint, split) pairs for a bf16 prompt-batch GEMM (M in the thousands): the ping-pong 256x256 kernel,
    the 8-wave 256x128 / 256x64 tiles, 128x128 tiled and stream-K, and the gemm_mid 256x128 / 128x256 /
    128x128 tiles with and without the interleaved ring (bench/prefill_plan_probe.py)."""
    out = [(4 << 8, 1), ((5 | 16) << 8, 1), ((6 | 16) << 8, 1), (1 << 8, 1), ((1 | 16) << 8, 1),
           ((1 | 128) << 8, 1), ((1 | 128) << 8, 2)]
    for t in (9, 12, 8):
        out += [((t | 16) << 8, 1)]
        if K % 64 == 0:
            out += [((t | 16 | 512) << 8, 1)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="65536,8192")
    ap.add_argument("--shapes", default="llama7b_tp8")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    H.reserve_workspace(dev, 256 << 20)
    for sname in a.shapes.split(","):
        for name, N, K in SHAPES[sname]:
            glu = name in ("gate_up", "up") and sname.startswith("llama")
            w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
            for M in [int(m) for m in a.m.split(",")]:
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                nout = N // 2 if glu else N
                y = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
                res = {"shape": sname, "layer": name, "M": M, "N": N, "K": K, "glu": glu}
                yl = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                res["hipblaslt_us"] = round(timeit(lambda i: torch.matmul(x, w.t(), out=yl), iters=a.iters), 1)
                for nt, s in prefill_candidates(M, N, K, glu):
                    try:
                        t = timeit(lambda i: H.linear(x, w, None, glu=glu, out=y, nt_hint=nt, split_hint=s),
                                   iters=a.iters)
                    except (ValueError, RuntimeError):
                        continue
                    res[f"{nt:#x}/s{s}"] = round(t, 1)
                ours = {k: v for k, v in res.items() if k.startswith("0x")}
                best = min(ours, key=ours.get)
                res["best"] = [best, ours[best], round(2 * M * N * K / ours[best] / 1e6, 1)]
                print(json.dumps(res), flush=True)
                del x, y, yl
            del w
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
