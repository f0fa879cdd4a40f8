"""In-situ A/B of decode GEMM plans: the autotuner times each projection alone (a HIP graph of calls of that one
GEMM), but in the decode step every GEMM sits between attention and add_norm launches. This builds the engine
with the tuned plans, then again with chosen projections forced to other plans (the process-wide tuning results
are edited before the engine installs them and captures its graphs), and compares the whole decode step:
64 requests x (128 prompt + 128 generated tokens), decode time per step from the engine's own counters.

usage: python bench/insitu_ab.py [--model gpt2-xl] [--reps 2]
"""
import argparse
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

VARIANTS = {  # label: {projection: (nt_hint, split)} at M = 64
    "gpt2-xl": [
        ("up mid64x32", {"up": ((14 | 32) << 8, 1)}),
        ("o,down mid64x32", {"o": ((14 | 32) << 8, 4), "down": ((14 | 32) << 8, 5)}),
        ("up,o,down mid64x32", {"up": ((14 | 32) << 8, 1), "o": ((14 | 32) << 8, 4), "down": ((14 | 32) << 8, 5)}),
        ("up dec64x64", {"up": ((4 | 32 | 1024) << 8, 1)}),
    ],
    "llama2-7b": [
        ("o,down mid64x96", {"o": ((15 | 32) << 8, 6), "down": ((15 | 32) << 8, 6)}),
        ("o,down dec64x64", {"o": ((4 | 32 | 1024) << 8, 4), "down": ((4 | 32 | 1024) << 8, 4)}),
        ("o,down mid64x128", {"o": ((11 | 32) << 8, 8), "down": ((11 | 32) << 8, 8)}),
        ("qkv mid64x96", {"qkv": ((15 | 32) << 8, 2)}),
    ],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl", choices=sorted(VARIANTS))
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from llmss_amd.engine import LLMEngine, build_model
    from llmss_amd.engine.sampling import SamplingParams
    from llmss_amd.ops import autotune as A

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = build_model(a.model, None, "bf16", dev, random_init=True)
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, model.cfg.vocab_size, (128,), generator=g).tolist() for _ in range(64)]
    sp = SamplingParams(max_new_tokens=128, temperature=1.0, top_p=0.95, top_k=50, ignore_eos=True)
    shapes = A.model_shapes(model)

    def run(label, forced):
        saved = {}
        for name, plan in forced.items():
            key = (64, shapes[name], str(dev))
            saved[key] = A._DONE[key]
            A._DONE[key] = (plan[0], plan[1]) + tuple(A._DONE[key][2:])
        try:
            eng = LLMEngine(model, max_num_seqs=64, max_batched_tokens=8192, max_model_len=264)
            plans = {n: "0x%x/s%d" % A._DONE[(64, shapes[n], str(dev))][:2] for n in ("qkv", "o", "up", "down")}
            eng.generate(prompts, sp)  # warm-up
            per = []
            for _ in range(a.reps):
                eng.stats["decode_time_s"] = 0.0
                eng.stats["decode_steps"] = 0
                eng.generate(prompts, sp)
                per.append(eng.stats["decode_time_s"] / max(1, eng.stats["decode_steps"]) * 1e3)
            print(json.dumps({"variant": label, "plans_m64": plans, "decode_ms_per_step": [round(x, 4) for x in per]}),
                  flush=True)
        finally:
            A._DONE.update(saved)
            eng = None
            gc.collect()
            torch.cuda.empty_cache()

    run("tuned", {})
    for label, forced in VARIANTS[a.model]:
        run(label, forced)
    run("tuned again", {})


if __name__ == "__main__":
    main()
