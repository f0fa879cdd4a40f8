"""QKV projection + RoPE + paged KV write: GEMM then rope_cache (two launches) vs the fused QKV GEMM epilogue
(one launch, ops/hip.py linear_qkv) for every fused-capable plan.

usage: python bench/qkv_epi_probe.py
Prints per config the unfused time (best slab plan + rope kernel) and the 3 fastest fused plans.
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402
from llmss_amd.ops import reference as R  # noqa: E402

CONFIGS = [  # name, M, K, nh, nkv, D, rot, style, bias
    ("llama7b tp1", 64, 4096, 32, 32, 128, 128, "neox", False),
    ("llama7b tp8", 512, 4096, 4, 4, 128, 128, "neox", False),
    ("gpt2-xl", 64, 1600, 25, 25, 64, 0, "none", True),
    ("llama13b tp8", 512, 5120, 5, 5, 128, 128, "neox", False),
    # the same Llama shapes with q/k head dims interleaved at load (neox pairs made adjacent, gptj-style
    # rotation in the epilogue): any tile width can rotate in-register
    ("llama7b tp1 il", 64, 4096, 32, 32, 128, 128, "gptj", False),
    ("llama7b tp8 il", 512, 4096, 4, 4, 128, 128, "gptj", False),
    ("llama13b tp8 il", 512, 5120, 5, 5, 128, 128, "gptj", False),
]


def main():
    dev = torch.device("cuda")
    H.reserve_workspace(dev)
    for name, M, K, nh, nkv, D, rot, style, has_b in CONFIGS:
        N = (nh + 2 * nkv) * D
        do_rope = style != "none"
        st = "gptj" if style == "gptj" else "neox"
        ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
        base = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        ws = [base.clone() for _ in range(ncopy)]
        b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16) if has_b else None
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        bs = 16
        kc = torch.zeros(-(-M // bs) + 1, nkv, bs, D, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        slots = torch.arange(M, device=dev)
        pos = torch.arange(M, device=dev) % 256
        cos, sin = R.rope_tables(4096, rot if do_rope else 64, 10000.0, dev)
        # unfused: best slab / finished plan of the GEMM + the rope kernel
        best_un = (float("inf"), None)
        for nt, s in [(0, 0)] + A.candidates(M, N, K, False, False):
            def f(i, nt=nt, s=s):
                q = H.linear(x, ws[i % ncopy], b, nt_hint=nt, split_hint=s, partial_ok=True)
                H.rope_cache(q, pos, cos, sin, kc, vc, slots, nh, nkv, D, rot, st, do_rope)
            try:
                f(0)
                torch.cuda.synchronize()
                t = A._time(f, 16)
            except (RuntimeError, ValueError):
                continue
            best_un = min(best_un, (t, (hex(nt), s)))
        fused = []
        for nt, s in A.qkv_epi_candidates(M, N, K, D, do_rope and st == "neox"):
            def g(i, nt=nt, s=s):
                if H.linear_qkv(x, ws[i % ncopy], b, pos, cos, sin, kc, vc, slots, nh, nkv, D, rot, st, do_rope,
                                nt_hint=nt, split_hint=s) is None:
                    raise RuntimeError("no fused plan")
            try:
                g(0)
                torch.cuda.synchronize()
                fused.append((A._time(g, 16), hex(nt), s))
            except (RuntimeError, ValueError):
                continue
        fused.sort()
        print(f"{name:15s} M={M:4d} N={N:5d} K={K:5d} unfused {best_un[0]:6.1f}us {best_un[1]} | fused: "
              + ", ".join(f"{t:.1f} ({nt}/s{s})" for t, nt, s in fused[:3]), flush=True)
        del ws


if __name__ == "__main__":
    main()
