"""Time one GEMM kernel configuration over a grid of (M, N, K, hint, split) - in-graph, HBM-streamed
weights - to separate per-k-step cost from fixed per-launch cost.
usage: python bench/gemm_scaling.py "M,N,K,hint,split" ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import timeit  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    dev = torch.device("cuda")
    for spec in sys.argv[1:]:
        M, N, K, hint, split = (int(v, 0) for v in spec.split(","))
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda i: H.linear(x, ws[i % ncopy], None, out=y, nt_hint=hint, split_hint=split), iters=30)
        tp = timeit(lambda i: H.linear(x, ws[i % ncopy], None, nt_hint=hint, split_hint=split, partial_ok=True),
                    iters=30)
        print(f"M={M} N={N} K={K} hint={hint:#x} split={split}: {t:.2f} us (slabs left to consumer: {tp:.2f} us), "
              f"{2 * M * N * K / t / 1e6:.0f} TF/s, weights {N * K * 2 / tp / 1e6:.2f} TB/s", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
