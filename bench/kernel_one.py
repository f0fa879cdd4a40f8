"""Run one non-GEMM hot kernel repeatedly on engine-shaped inputs (for rocprofv3 counter passes).

usage: python bench/kernel_one.py decode|prefill|sample|add_norm|rope [--iters 100]
  decode   paged decode attention, Llama-2-7B TP=1 shape: B=64, 32 heads x 128, context 192
           (KV rotated over copies larger than the Infinity Cache, as a decode step streams it)
  prefill  flash prefill attention, 8 prompts x 2048 tokens, 32 heads x 128
  sample   temperature / top-k / top-p sampler, B=64 rows of a 32000 vocabulary
  add_norm fused residual add + RMSNorm, 64 x 4096
  rope     RoPE + paged KV write, 64 tokens, 32 heads x 128
  gemm_big prefill GEMM (the 256 x 256 8-wave kernel), Llama-2-7B QKV at 8192 prompt tokens: 8192 x 12288 x 4096
  cand     vocab-parallel candidate sampler at TP=8 rows: cand_topk on a [512, 4000] shard + sample_cand over
           8 gathered groups
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402
from llmss_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    nh, nkv, D, bs = 32, 32, 128, 16
    if a.kernel == "decode":
        B, ctx = 64, 192
        maxb = ctx // bs
        nb = B * maxb
        ncopy = max(2, int(700e6 // (2 * nb * nkv * bs * D * 2)) + 1)
        kcs = [torch.randn(nb, nkv, bs, D, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        vcs = [torch.randn_like(kcs[0]) for _ in range(ncopy)]
        bt = torch.arange(nb, device=dev, dtype=torch.int32).view(B, maxb)
        cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        q = torch.randn(B, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
        out = torch.empty(B, nh * D, device=dev, dtype=torch.bfloat16)

        def f(i):
            H.attn_decode(q, kcs[i % ncopy], vcs[i % ncopy], bt, cl, nh, nkv, D, D ** -0.5, ctx, out=out)
    elif a.kernel == "prefill":
        S, nseq = 2048, 8
        T = S * nseq
        qkv = torch.randn(T, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
        cu = torch.arange(0, T + 1, S, device=dev, dtype=torch.int32)
        out = torch.empty(T, nh * D, device=dev, dtype=torch.bfloat16)

        def f(i):
            H.attn_prefill(qkv, cu, S, nh, nkv, D, D ** -0.5, out=out)
    elif a.kernel == "sample":
        B, V = 64, 32000
        lg = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
        t = torch.ones(B, device=dev)
        k = torch.full((B,), 50, dtype=torch.int32, device=dev)
        p = torch.full((B,), 0.95, device=dev)
        sd = torch.arange(B, dtype=torch.int64, device=dev)

        def f(i):
            H.sample(lg, t, k, p, sd)
    elif a.kernel == "add_norm":
        x = torch.randn(64, 4096, device=dev).to(torch.bfloat16)
        r = torch.randn_like(x)
        w = torch.ones(4096, device=dev, dtype=torch.bfloat16)

        def f(i):
            H.add_norm(x, w, None, 1e-5, True, r)
    elif a.kernel == "rope":
        B, maxb = 64, 16
        qkv = torch.randn(B, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
        kc = torch.zeros(B * maxb, nkv, bs, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        pos = torch.full((B,), 100, dtype=torch.int64, device=dev)
        slots = torch.arange(B, dtype=torch.int64, device=dev) * (maxb * bs) + 100
        cos, sin = R.rope_tables(4096, D, 10000.0, dev)

        def f(i):
            H.rope_cache(qkv, pos, cos, sin, kc, vc, slots, nh, nkv, D, D, "neox")
    elif a.kernel == "gemm_big":
        M, N, K = 8192, 12288, 4096
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def f(i):
            H.linear(x, w, None, out=y)
    elif a.kernel == "cand":
        B, vl, tp = 512, 4000, 8
        lg = (torch.randn(B, vl, device=dev) * 3).to(torch.bfloat16)
        t = torch.ones(B, device=dev)
        k = torch.full((B,), 50, dtype=torch.int32, device=dev)
        p = torch.full((B,), 0.95, device=dev)
        sd = torch.arange(B, dtype=torch.int64, device=dev)

        def f(i):
            pack = H.cand_topk(lg, 0, vl * tp, t, k)
            H.sample_cand(torch.cat([pack] * tp, -1), H.CAND_KC, t, k, p, sd)
    else:
        raise SystemExit(f"unknown kernel {a.kernel}")
    for i in range(a.iters):
        f(i)
    torch.cuda.synchronize()
    print(f"{a.kernel}: {a.iters} launches", flush=True)


if __name__ == "__main__":
    main()
