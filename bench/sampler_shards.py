"""Full-row sampler (sample_v3, one workgroup per row) against the candidate kernels over S column shards of the
same row (cand_topk grid.y = S, then sample_cand on the union: exact for greedy and top-k <= 64 rows), per call at
B rows, in HIP graphs of 20 calls. usage: python bench/sampler_shards.py [B]"""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.ops import hip as H  # noqa: E402


def timed(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(n):
            f()
    best = float("inf")
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / n)
    return round(best, 2)


def main():
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    for V, Vp in ((32000, 32000), (50257, 50304)):
        logits = (torch.randn(B, Vp, device=dev) * 2.0).to(torch.bfloat16)
        for mode in ("greedy", "topk50_topp0.95"):
            temp = torch.full((B,), 0.0 if mode == "greedy" else 1.0, device=dev)
            topk = torch.full((B,), 50 if "topk" in mode else 0, dtype=torch.int32, device=dev)
            topp = torch.full((B,), 0.95 if "topp" in mode else 1.0, device=dev)
            seeds = torch.arange(B, dtype=torch.int64, device=dev)
            out = torch.empty(B, dtype=torch.int64, device=dev)
            res = {"B": B, "V": V, "mode": mode,
                   "v3_us": timed(lambda: H.sample(logits, temp, topk, topp, seeds, vocab=V, out=out))}
            ref = out.clone()
            for S in (2, 4, 8, 16):
                if -(-Vp // S) > H.CAND_MAX_SHARD:
                    continue
                pack = torch.empty(B, S * 2 * H.CAND_KC, dtype=torch.float32, device=dev)
                o2 = torch.empty(B, dtype=torch.int64, device=dev)

                def f():
                    H.cand_topk(logits, 0, V, temp, topk, out=pack, shards=S)
                    H.sample_cand(pack, H.CAND_KC, temp, topk, topp, seeds, out=o2)
                res[f"s{S}_us"] = timed(f)
                res[f"s{S}_topk_us"] = timed(lambda: H.cand_topk(logits, 0, V, temp, topk, out=pack, shards=S))
                res[f"s{S}_same"] = bool(torch.equal(o2, ref))
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
