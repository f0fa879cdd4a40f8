"""Sampler kernel time per call (B rows) by vocab, logit spread and sampling mode."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = int(os.environ.get("B", "64"))
    for V in (32000, 50257, 50304):
        for spread in (0.5, 1.0, 5.0):
            logits = (torch.randn(B, V, device=dev) * spread).to(torch.bfloat16)
            for mode in ("greedy", "topk50_topp0.95", "topp0.95"):
                temp = torch.full((B,), 0.0 if mode == "greedy" else 1.0, device=dev)
                topk = torch.full((B,), 50 if "topk" in mode else 0, dtype=torch.int32, device=dev)
                topp = torch.full((B,), 0.95 if "topp" in mode else 1.0, device=dev)
                seeds = torch.arange(B, dtype=torch.int64, device=dev)
                out = torch.empty(B, dtype=torch.int64, device=dev)
                f = lambda: H.sample(logits, temp, topk, topp, seeds, vocab=V, out=out)  # noqa: E731
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    for _ in range(20):
                        f()
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                g.replay()
                e.record()
                e.synchronize()
                print(json.dumps({"B": B, "V": V, "spread": spread, "mode": mode,
                                  "us": round(s.elapsed_time(e) / 20 * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
