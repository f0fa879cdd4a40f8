"""Prefill (flash) attention throughput: v1 vs v2 kernels, causal, packed sequences.

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
            for v in (1, 2):
                H.lib().attn_prefill_set_version(v)
                for _ in range(3):
                    H.attn_prefill(qkv, cu, S, nh, nkv, D, D ** -0.5, out=out)
                torch.cuda.synchronize()
                it = 10
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
            H.lib().attn_prefill_set_version(2)
            res["max_diff_v1_v2"] = float((outs[1].float() - outs[2].float()).abs().max())
            print(res, flush=True)


if __name__ == "__main__":
    main()
