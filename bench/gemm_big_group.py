"""Prefill GEMM (256x256 big-tile kernel): launch-order tile group height vs time.
usage: python bench/gemm_big_group.py [--m 8192] [--groups 1,2,4,8,16]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import timeit  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--groups", default="1,2,4,8,16")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name, N, K, glu in (("qkv", 12288, 4096, False), ("gate_up", 22016, 4096, True), ("down", 4096, 11008, False)):
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        x = torch.randn(a.m, K, device=dev).to(torch.bfloat16)
        row = {"layer": name}
        for gm in map(int, a.groups.split(",")):
            H.lib().gemm_big_set_group(gm)
            t = timeit(lambda i: H.linear(x, w, None, glu=glu, nt_hint=4 << 8, split_hint=1))
            row[f"g{gm}_us"] = round(t, 1)
            row[f"g{gm}_TF"] = round(2 * a.m * N * K / t / 1e6, 1)
        H.lib().gemm_big_set_group(4)
        print(row, flush=True)


if __name__ == "__main__":
    main()
