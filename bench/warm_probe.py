"""Decode GEMMs with HBM-cold vs Infinity-Cache-resident weights: is a decode GEMM bound by the HBM stream or
by its own launch / pipeline structure?

usage: python bench/warm_probe.py
Per shape: the autotuner's best plan timed (HIP graph) rotating over > 600 MB of weight copies (every call
streams from HBM, as in a decode step) and on one copy (after the first call the weights sit in the 256 MB
Infinity Cache). A large cold/warm gap means the kernel would go faster with its weights already on chip
(e.g. fetched in an idle phase of a preceding kernel); a small gap means the kernel structure is the limit.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import autotune as A  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402

SHAPES = [  # name, M, N, K, glu, partial
    ("llama7b qkv", 64, 12288, 4096, False, True),
    ("llama7b o", 64, 4096, 4096, False, True),
    ("llama7b gate_up", 64, 22016, 4096, True, False),
    ("llama7b down", 64, 4096, 11008, False, True),
    ("llama7b_tp8 qkv", 512, 1536, 4096, False, True),
    ("llama7b_tp8 gate_up", 512, 2752, 4096, True, False),
    ("llama7b_tp8 down", 512, 4096, 1376, False, False),
    ("gpt2xl fc", 64, 6400, 1600, False, False),
    ("gpt2xl proj", 64, 1600, 6400, False, True),
]


def main():
    dev = torch.device("cuda")
    H.reserve_workspace(dev)
    print(f"{'shape':22s} {'MB':>6s} {'plan':>12s} {'cold us':>8s} {'TB/s':>5s} {'warm us':>8s} {'TB/s':>5s}", flush=True)
    for name, M, N, K, glu, partial in SHAPES:
        sh = A.GemmShape(N, K, glu, False, partial, "none")
        nt, s, t_cold, _ = A.tune_shape(M, sh, dev)
        r = A.tune_shape(M, sh, dev, cands=[(nt, s)] if nt else [], copies=1)
        t_warm = r[2] if nt and r[0] == nt else (r[3] if not nt else min(r[2], r[3]))
        mb = N * K * 2 / 1e6
        print(f"{name:22s} {mb:6.1f} {hex(nt) + '/s' + str(s):>12s} {t_cold:8.1f} {mb / t_cold:5.2f} "
              f"{t_warm:8.1f} {mb / t_warm:5.2f}", flush=True)


if __name__ == "__main__":
    main()
