"""Prefill (flash) attention throughput: v1 / v2 / v3 kernels, causal, packed sequences.

usage: python bench/attn_prefill_bench.py [--S 128,2048,4096,8192] [--heads 32:32:128,32:8:128,64:8:128,16:16:256,25:25:64]
Each config runs `tokens` = max(S, 16384) total tokens (several sequences of length S); TFLOP/s counts
the causal half only: 4 * sum(S_i^2 / 2) * D * nh.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", default="128,2048,4096,8192")
    ap.add_argument("--heads", default="32:32:128,32:8:128,64:8:128,16:16:256,25:25:64")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--versions", default="1,2,3:4,3:8", help="kernel version[:waves per workgroup]")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for spec in a.heads.split(","):
        nh, nkv, D = map(int, spec.split(":"))
        for S in map(int, a.S.split(",")):
            nseq = max(1, a.tokens // S)
            T = nseq * S
            qkv = torch.randn(T, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
            cu = torch.arange(0, T + 1, S, device=dev, dtype=torch.int32)
            out = torch.empty(T, nh * D, device=dev, dtype=torch.bfloat16)
            flops = 4 * nseq * (S * S / 2) * D * nh
            res = {"nh": nh, "nkv": nkv, "D": D, "S": S, "nseq": nseq}
            outs = {}
            vers = a.versions.split(",")
            for v in vers:
                H.lib().attn_prefill_set_version(int(v.split(":")[0]))
                H.lib().attn_prefill_set_waves(int(v.split(":")[1]) if ":" in v else 0)
                for _ in range(3):
                    H.attn_prefill(qkv, cu, S, nh, nkv, D, D ** -0.5, out=out)
                torch.cuda.synchronize()
                it = a.iters
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(it):
                    H.attn_prefill(qkv, cu, S, nh, nkv, D, D ** -0.5, out=out)
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1e3 / it
                res[f"v{v}_us"] = round(us, 1)
                res[f"v{v}_TFs"] = round(flops / us / 1e6, 1)
                outs[v] = out.clone()
            H.lib().attn_prefill_set_version(3)
            H.lib().attn_prefill_set_waves(0)
            # fp32 reference on the first sequence (causal softmax(QK^T/sqrt(D))V) for every version
            S0 = min(S, 2048)
            x = qkv[:S0].float()
            q = x[:, :nh * D].view(S0, nh, D).transpose(0, 1)
            k = x[:, nh * D:(nh + nkv) * D].view(S0, nkv, D).transpose(0, 1).repeat_interleave(nh // nkv, 0)
            vv = x[:, (nh + nkv) * D:].view(S0, nkv, D).transpose(0, 1).repeat_interleave(nh // nkv, 0)
            sc = (q @ k.transpose(1, 2)) * D ** -0.5
            sc = sc.masked_fill(torch.triu(torch.ones(S0, S0, dtype=torch.bool, device=dev), 1), float("-inf"))
            ref = (sc.softmax(-1) @ vv).transpose(0, 1).reshape(S0, nh * D)
            for v in vers:
                res[f"v{v}_err"] = round(float((outs[v][:S0].float() - ref).abs().max()), 5)
            print(res, flush=True)


if __name__ == "__main__":
    main()
