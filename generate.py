"""Offline tensor-parallel generation CLI (API-compatible with the reference ``generate.py``).

Same flags, defaults, validation and the same three stdout lines as the reference
(``generate.py:21-40,192-196``); launched with ``torchrun --nproc_per_node N generate.py ...``
(one rank per GPU, RCCL) or plain ``python generate.py ...`` (TP=1, GPU or CPU).

Deliberate fixes: TP=1 works (Q2); temperature/top-k/top-p are actually applied
(Q1); prompts are not padded, each sequence has its own length and positions (Q3); load time and
generation throughput are reported on extra lines after the original three (Q12).
``--use_cache`` absent keeps the reference's recompute mode (the whole prefix is re-run every
token, generate.py:146-190) over the same kernels.
"""
from __future__ import annotations

import json
import os
import sys
import time
from argparse import ArgumentParser

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def get_args(argv=None):
    parser = ArgumentParser()
    parser.add_argument("--pretrained_model_path", type=str, required=True)
    parser.add_argument("--prompts", type=str, nargs="+", required=True)
    parser.add_argument("--max_new_tokens", type=int, default=20)
    parser.add_argument("--is_greedy", action="store_true")
    parser.add_argument("--temperature", type=float, default=1.0, help="If you don't wanna use this, set to 1.0")
    parser.add_argument("--top_p", type=float, default=0.95, help="If you don't wanna use this, set to 1.0")
    parser.add_argument("--top_k", type=int, default=50, help="If you don't wanna use this, set to 0")
    parser.add_argument("--use_cache", action="store_true")
    # additions
    parser.add_argument("--dtype", type=str, default=None, help="bf16 (GPU default) | fp32 (CPU default)")
    parser.add_argument("--fp8", action="store_true", help="fp8-e4m3 weights (per-channel scales)")
    parser.add_argument("--seed", type=int, default=None)
    parser.add_argument("--device", type=str, default=None, help="cuda | cpu (default: cuda if available)")
    parser.add_argument("--json_metrics", action="store_true")
    return parser.parse_args(argv)


def recompute_generate(model, prompts, params, eos):
    """Reference no-cache mode: every step re-runs the full prefix of every sequence."""
    from llmss_amd import ops
    from llmss_amd.engine.sampling import step_seed
    from llmss_amd.models.decoder import StepInput

    dev = model.device
    seqs = [list(p) for p in prompts]
    outs = [[] for _ in prompts]
    done = [False] * len(prompts)
    nokv = [(None, None)] * model.cfg.num_layers
    maxlen = model.cfg.max_position_embeddings
    for step in range(params.max_new_tokens):
        live = [i for i in range(len(seqs)) if not done[i]]
        if not live:
            break
        cur = [seqs[i][-maxlen:] for i in live]  # sliding window like the reference (generate.py:176-178)
        lens = [len(c) for c in cur]
        ids = torch.tensor([t for c in cur for t in c], dtype=torch.int64, device=dev)
        pos = torch.cat([torch.arange(n, dtype=torch.int64) for n in lens]).to(dev)
        cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), dtype=torch.int32, device=dev)
        inp = StepInput("prefill", ids, pos, torch.full_like(pos, -1), cu_seqlens=cu, max_seqlen=max(lens),
                        last_idx=(cu[1:] - 1).to(torch.int64))
        logits = model(inp, nokv)
        n = len(live)
        temp = torch.full((n,), params.k_temperature, dtype=torch.float32, device=dev)
        topk = torch.full((n,), params.k_top_k, dtype=torch.int32, device=dev)
        topp = torch.full((n,), params.k_top_p, dtype=torch.float32, device=dev)
        seeds = torch.tensor([step_seed(params.resolved_seed() + i, step) for i in live], dtype=torch.int64, device=dev)
        tok = ops.sample(logits, temp, topk, topp, seeds, vocab=model.cfg.vocab_size).tolist()
        for i, t in zip(live, tok):
            seqs[i].append(t)
            outs[i].append(t)
            if eos is not None and t == eos:
                done[i] = True
    return outs


def main(argv=None):
    args = get_args(argv)
    assert args.max_new_tokens > 0, "Value of max_new_tokens should be over than 0."
    assert 0.0 < args.temperature <= 1.0, "Value of temperature is not valid."
    assert 0.0 < args.top_p <= 1.0, "Value of top_p is not valid."
    assert args.top_k >= 0, "Value of top_k is not valid."

    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed
    from llmss_amd.utils.tokenizer import encode, load_tokenizer

    tp, rank, world_size = initialize_distributed()
    start_time = time.time()
    if args.device:
        device = torch.device(args.device if args.device != "cuda" else f"cuda:{torch.cuda.current_device()}")
    else:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dtype = args.dtype or ("bf16" if device.type == "cuda" else "fp32")
    tp.barrier()
    model = build_model(args.pretrained_model_path, tp, dtype, device, fp8=args.fp8)
    tokenizer = load_tokenizer(args.pretrained_model_path, model.cfg.vocab_size)
    load_done = time.time()

    seed = args.seed
    if seed is None:  # one seed for all ranks so they sample identically
        seed = tp.broadcast_object(int.from_bytes(os.urandom(4), "little") if rank == 0 else None)
    params = SamplingParams(max_new_tokens=args.max_new_tokens, is_greedy=args.is_greedy,
                            temperature=args.temperature, top_p=args.top_p, top_k=args.top_k, seed=seed)
    eos = getattr(tokenizer, "eos_token_id", None)
    prompts = [encode(tokenizer, p) for p in args.prompts]
    max_len = model.cfg.max_position_embeddings
    prompts = [p[-max(1, max_len - 1):] for p in prompts]  # left truncation (reference tokenizer settings)

    t0 = time.time()
    if args.use_cache:
        engine = LLMEngine(model, max_num_seqs=max(1, len(prompts)), eos_token_id=eos)
        per = [SamplingParams(**{**params.__dict__, "seed": seed + i}) for i in range(len(prompts))]
        outputs = engine.generate(prompts, per)
    else:
        outputs = recompute_generate(model, prompts, params, eos)
    gen_s = time.time() - t0

    if rank == 0:
        end_time = time.time()
        print(f"elapsed time: {end_time - start_time}")
        print(f"prompts: {args.prompts}")
        print(f"continuations: {[tokenizer.decode(o) for o in outputs]}")
        n = sum(len(o) for o in outputs)
        print(f"load time: {load_done - start_time:.3f} s, generation: {gen_s:.3f} s, "
              f"{n} tokens, {n / max(gen_s, 1e-9):.1f} tokens/s (tp={world_size}, {device.type}, {dtype})")
        if args.json_metrics:
            print(json.dumps({"load_s": load_done - start_time, "generate_s": gen_s, "tokens": n,
                              "tokens_per_s": n / max(gen_s, 1e-9), "tp": world_size}))
    return outputs


if __name__ == "__main__":
    main()
