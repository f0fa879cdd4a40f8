"""Decode-attention micro-benchmark: paged KV read bandwidth per configuration.

usage: python bench/attn_bench.py [--B 64] [--ctx 192,1024] [--heads 32:32,32:8] [--bs 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--ctx", default="192,1024")
    ap.add_argument("--heads", default="32:32,32:8")
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--random-pages", action="store_true", help="scatter pages (default: engine-like sequential)")
    ap.add_argument("--splits", default="", help="context splits to sweep (default: the engine's decode_splits)")
    ap.add_argument("--unrolls", default="1,2,4,11,12,14")
    ap.add_argument("--bs", type=int, default=16, help="KV cache block (page) size in tokens")
    ap.add_argument("--rotate-mb", type=float, default=700,
                    help="K/V copies rotated over at least this many MB (default: past the 256 MiB Infinity Cache; "
                         "the decode step's own working set is ~20 GB)")
    a = ap.parse_args()
    dev, bs, D = "cuda", a.bs, a.D
    for hk in a.heads.split(","):
        nh, nkv = map(int, hk.split(":"))
        for ctx in map(int, a.ctx.split(",")):
            maxb = (ctx + bs - 1) // bs
            nb = a.B * maxb
            kv_bytes = 2 * a.B * ctx * nkv * D * 2
            ncopy = max(1, int(a.rotate_mb * 1e6 // kv_bytes) + 1)  # rotate copies past the 256 MiB Infinity Cache
            kcs = [torch.randn(nb, nkv, bs, D, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
            vcs = [torch.randn_like(kcs[0]) for _ in range(ncopy)]
            pages = torch.randperm(nb, device=dev) if a.random_pages else torch.arange(nb, device=dev)
            bt = pages.view(a.B, maxb).to(torch.int32)
            cl = torch.full((a.B,), ctx, dtype=torch.int32, device=dev)
            q = torch.randn(a.B, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
            out = torch.empty(a.B, nh * D, device=dev, dtype=torch.bfloat16)
            res = {"B": a.B, "nh": nh, "nkv": nkv, "ctx": ctx, "MB": round(kv_bytes / 1e6, 1)}
            for u, sp in [(u, sp) for u in map(int, a.unrolls.split(",")) for sp in
                          (map(int, a.splits.split(",")) if a.splits else [0])]:
                H.lib().attn_decode_set_unroll(u)
                spl = None
                if sp:
                    ps = -(-ctx // sp)
                    ps = -(-ps // bs) * bs
                    spl = (-(-ctx // ps), ps)
                it = [0]

                def f():
                    i = it[0] = (it[0] + 1) % ncopy
                    H.attn_decode(q, kcs[i], vcs[i], bt, cl, nh, nkv, D, D ** -0.5, ctx, out=out, splits=spl)
                for _ in range(5):
                    f()
                torch.cuda.synchronize()
                # 50 calls in one HIP graph (as the decode graphs run it): no host launch cost in the time
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    for _ in range(50):
                        f()
                g.replay()
                torch.cuda.synchronize()
                us = float("inf")
                for _ in range(3):
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    g.replay()
                    e.record()
                    torch.cuda.synchronize()
                    us = min(us, s.elapsed_time(e) * 1e3 / 50)
                del g
                tag = f"u{u}" + (f"s{sp}" if sp else "")
                res[f"{tag}_us"] = round(us, 2)
                res[f"{tag}_TBps"] = round(kv_bytes / us / 1e6, 2)
            H.lib().attn_decode_set_unroll(0)  # back to the default
            print(res, flush=True)


if __name__ == "__main__":
    main()
