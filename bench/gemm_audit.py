"""Run every autotuner candidate once per (shape, M) with a synchronize after each launch and the
configuration printed (flushed) BEFORE it runs: if a launch faults, the last line names it.

usage: python bench/gemm_audit.py --model llama2-70b --tp 8 [--fp8] [--m 1,16,24,64,128,256,512]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmss_amd.models.config import get_preset  # noqa: E402
from llmss_amd.models.weights import shard_plan  # noqa: E402
from llmss_amd.ops import hip as H  # noqa: E402
from llmss_amd.ops.autotune import candidates  # noqa: E402


def shapes(cfg, tp):
    p = shard_plan(cfg, tp, 0)
    D = cfg.head_dim
    up = 2 * p.F_l if cfg.gated_mlp else p.F_l
    return [("qkv", (p.nh_l + 2 * p.nkv_l) * D, cfg.hidden_size, False, True),
            ("o", cfg.hidden_size, p.nh_l * D, False, True),
            ("up", up, cfg.hidden_size, cfg.gated_mlp, True),
            ("down", cfg.hidden_size, p.F_l, False, True),
            ("head", p.v_l, cfg.hidden_size, False, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--m", default="1,16,24,64,128,256,512")
    a = ap.parse_args()
    cfg = get_preset(a.model)
    dev = "cuda"
    for name, N, K, glu, quant in shapes(cfg, a.tp):
        part = name in ("qkv", "o", "down")  # the autotuner times these as split-K producers
        fp8 = a.fp8 and quant
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        sc = None
        if fp8:
            w, sc = H.quant_fp8_rows(w)
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            for nt, s in [(0, 0)] + candidates(M, N, K, glu, fp8):
                print(f"{name} N={N} K={K} glu={glu} fp8={fp8} M={M} nt={nt:#x} s={s}", flush=True)
                try:
                    H.linear(x, w, None, "none", glu, sc, nt_hint=nt, split_hint=s, partial_ok=part)
                except (ValueError, RuntimeError) as e:
                    print("  rejected:", e, flush=True)
                torch.cuda.synchronize()
        del w
    print("audit ok", flush=True)


if __name__ == "__main__":
    main()
