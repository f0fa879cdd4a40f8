"""add + norm at decode sizes, timed as the decode graphs run it (calls captured into one HIP graph, ops/autotune.py
_time): the launch against the ~1.85 us of a minimal dependent kernel (bench/launch_floor.hip).

usage: python bench/addnorm_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for name, M, N, rms, bias, S in [("llama7b", 64, 4096, True, False, 0), ("llama7b", 64, 4096, True, False, 4),
                                     ("llama7b", 64, 4096, True, False, 8), ("gpt2xl", 64, 1600, False, True, 0),
                                     ("gpt2xl", 64, 1600, False, True, 2), ("llama7b_tp8", 512, 4096, True, False, 0)]:
        w = torch.randn(N, device=dev).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16) if bias else None
        res = torch.randn(M, N, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if S:
            x = H.PartialSum(torch.randn(S, M, N, device=dev), S, M, N, None, dev)
        else:
            x = torch.randn(M, N, device=dev).to(torch.bfloat16)

        def f(i):
            H.add_norm(x, w, b, 1e-5, rms, res, out=y)
        f(0)
        torch.cuda.synchronize()
        t = A._time(f, 64)
        print(json.dumps({"shape": name, "M": M, "N": N, "slabs": S, "rms": rms, "us": round(t, 2)}), flush=True)


if __name__ == "__main__":
    main()
