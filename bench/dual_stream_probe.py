"""Does a TP=1 decode step run faster as two half-batch layer chains on two HIP streams?

GPT-2-XL / Llama-2-7B decode kernels at batch 64 are latency-bound (ramp, drain and fixed costs of every launch;
profiles/r3_bench). Two independent half-batch chains on two streams can fill each other's gaps; the weights are
read twice, but the second read of a 5-20 MB projection finds it in the 256 MiB Infinity Cache.

Measures (HIP-graph replays, random-init weights, every sequence at context CTX):
  one:  hidden_states of B rows + LM head, one stream
  two:  rows [0, B/2) on the capture stream, rows [B/2, B) on a forked stream, joined at the end
usage: MODEL=gpt2-xl B=64 CTX=192 python bench/dual_stream_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM, StepInput
    from llmss_amd.models.weights import random_weights
    from llmss_amd.ops import hip as H
    from llmss_amd.ops.autotune import tune_model

    dev = torch.device("cuda", 0)
    name = os.environ.get("MODEL", "gpt2-xl")
    B, ctx, bs = int(os.environ.get("B", "64")), int(os.environ.get("CTX", "192")), 16
    cfg = get_preset(name)
    w = random_weights(cfg, 1, 0, device=dev, dtype=torch.bfloat16, seed=0)
    m = DecoderLM(cfg, w)
    H.reserve_workspace(dev, decode_rows=B, nh=m.plan.nh_l, D=cfg.head_dim)
    tune_model(m, [B // 2, B])
    nbps = -(-(ctx + 1) // bs)
    kv = m.allocate_kv_cache(B * nbps + 1, bs)
    bt = torch.arange(B * nbps, device=dev, dtype=torch.int32).view(B, nbps)
    ids = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    pos = torch.full((B,), ctx, device=dev, dtype=torch.int64)
    slots = (bt[:, ctx // bs].long() * bs + ctx % bs).contiguous()
    cl = torch.full((B,), ctx + 1, device=dev, dtype=torch.int32)

    def step(r0, r1):
        n = r1 - r0
        return StepInput("decode", ids[r0:r1], pos[r0:r1], slots[r0:r1], block_tables=bt[r0:r1],
                         ctx_lens=cl[r0:r1], max_ctx=ctx + 1,
                         decode_splits=H.decode_splits(n, m.plan.nkv_l, ctx + 1, bs))

    def fwd(inp):
        h = m.hidden_states(inp, kv)
        return m.local_logits(h)

    s_one, s_a, s_b = step(0, B), step(0, B // 2), step(B // 2, B)
    side = torch.cuda.Stream(device=dev)

    def one():
        fwd(s_one)

    def two():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        fwd(s_a)
        with torch.cuda.stream(side), H.workspace_slot(1):
            fwd(s_b)
        cur.wait_stream(side)

    res = {"model": name, "batch": B, "ctx": ctx}
    for tag, fn in (("one", one), ("two", two), ("one_again", one)):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            fn()
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 10 * 1e3)
        res[tag + "_us"] = round(best, 1)
        del g
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
