"""Headline benchmark: output tokens/s (node) + p50 latency for batched generation.

Config (BASELINE.json): Llama-2-7B with tensor parallelism TP = N (one process per GPU, RCCL over
xGMI; TP=8 at N=8) - or ``--model gpt2-xl`` for the GPT-2-XL TP=1 configuration. Random-init
weights of the exact architecture and synthetic prompt token ids (no network, no checkpoints).

A "step" = one complete batched generation through the serving engine: ``batch`` synthetic
prompts of ``--prompt-len`` tokens, prefill + ``--gen-len`` decode tokens each (continuous-
batching scheduler, paged KV cache, HIP-graph decode, on-device sampling with the reference's
default temperature=1.0 / top_p=0.95 / top_k=50). Weak scaling: the global batch is
``--batch-per-gpu * N``. ``value`` = total generated tokens / wall time over all ranks (max).

Launch: ``python bench.py`` (N=1) or ``torchrun --nproc-per-node N bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="paged KV cache storage: bf16, or fp8 e4m3 rows with per-row scales")
    ap.add_argument("--greedy", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--secondary", default="gpt2-xl",
                    help="second headline model timed after the first (TP=1 per GPU, data-parallel over N GPUs); "
                         "'' or 'none' to skip")
    ap.add_argument("--simulate-tp", type=int, default=0,
                    help="dev tool: one process computes rank 0 of a TP=N shard plan with no communication "
                         "(per-rank compute time at TP=N shapes; not a headline number)")
    ap.add_argument("--sim-comm", default="",
                    help="with --simulate-tp: model each all-reduce / all-gather as LAT_US,GBPS (latency + bytes / "
                         "algorithmic bandwidth, a spin kernel on the collective's stream) to measure comm overlap")
    args = ap.parse_args()

    from llmss_amd.parallel.dist import TPGroup, initialize_distributed

    tp, rank, world = initialize_distributed()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.simulate_tp > 1:
        if world != 1:
            raise SystemExit("--simulate-tp runs in a single process")
        sim = tuple(float(v) for v in args.sim_comm.split(",")) if args.sim_comm else None
        tp = TPGroup(0, args.simulate_tp, fake=True, sim_comm=sim)
        tp.replicate_gather = True  # the gathered candidates / logits have their TP=N width

    def progress(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    res = run_config(args, args.model, tp, args.batch_per_gpu * max(world, args.simulate_tp), progress)
    if args.secondary not in ("", "none") and args.simulate_tp <= 1 and args.secondary != args.model:
        # second BASELINE headline config (GPT-2-XL TP=1, 25 heads: no TP split), driver-timed in the same run;
        # with N GPUs every rank serves its own TP=1 replica (data parallel) and the node total is reported
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        res["secondary"] = run_config(args, args.secondary, tp, args.batch_per_gpu * world, progress, dp=True)
    if rank == 0:
        print(json.dumps(res))
    if tp.is_real:
        torch.distributed.destroy_process_group()


def run_config(args, model_name, tp, batch, progress, dp=False):
    """Build ``model_name`` on ``tp`` (``dp``: an independent TP=1 replica per rank), warm up, time
    ``args.steps`` batched generations; returns the JSON dict."""
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    world = args.gpus
    # GPU: this rank's device. CPU (no GPU): the PyTorch reference path over gloo - a functional rehearsal
    # of the multi-rank bench (tests/test_bench_dist.py), not a performance number
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    local_batch = batch // world if dp else batch
    model = build_model(model_name, tp if not dp else None, "bf16", dev, fp8=args.fp8, random_init=True)
    max_len = min(model.cfg.max_position_embeddings, max(256, args.prompt_len + args.gen_len))
    eng = LLMEngine(model, max_num_seqs=local_batch, max_batched_tokens=max(8192, local_batch * args.prompt_len),
                    block_size=16, max_model_len=max_len, use_graphs=not args.no_graphs, kv_dtype=args.kv_dtype)
    rng = np.random.default_rng(1234 + (tp.rank if dp else 0))
    V = model.cfg.vocab_size

    def prompts():
        return [rng.integers(0, V, args.prompt_len).tolist() for _ in range(local_batch)]

    def params():
        return SamplingParams(max_new_tokens=args.gen_len, is_greedy=args.greedy, temperature=1.0, top_p=0.95,
                              top_k=50, ignore_eos=True, seed=7)

    def one_step():
        for p in prompts():
            eng.add_request(p, params())
        n = 0
        while eng.has_unfinished():
            n += len(eng.step())
        reqs = eng.pop_finished()
        return n, [r.metrics() for r in reqs]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def barrier():
        if world > 1 and args.simulate_tp <= 1:
            torch.distributed.barrier()

    progress(f"engine ready: {model.cfg.model_type} {'dp' if dp else 'tp'}={world} batch={batch} "
             f"kv_blocks={eng.num_blocks} graphs={sorted({b for b, _ in eng.graphs})}")
    if eng.tuned:
        mx = max(m for _, m in eng.tuned)
        progress("autotuned GEMMs at M=%d: " % mx + ", ".join(
            f"{n} {nt:#x}/s{sp} {t:.1f}us (static {t0:.1f})" for (n, m), (nt, sp, t, t0) in sorted(eng.tuned.items())
            if m == mx))
    for i in range(args.warmup):
        t = time.perf_counter()
        one_step()
        progress(f"warmup {i}: {time.perf_counter() - t:.3f}s")
    barrier()
    sync()
    t0 = time.perf_counter()
    total, mets = 0, []
    for i in range(args.steps):
        n, m = one_step()
        total += n
        mets.extend(m)
        progress(f"step {i}: {n} tokens, {time.perf_counter() - t0:.3f}s elapsed")
    sync()
    barrier()
    el = time.perf_counter() - t0
    if world > 1 and args.simulate_tp <= 1:  # slowest rank's clock; node total of generated tokens
        t = torch.tensor([el, float(total)], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t[:1], op=torch.distributed.ReduceOp.MAX)
        if dp:
            torch.distributed.all_reduce(t[1:], op=torch.distributed.ReduceOp.SUM)
        el, total = float(t[0].item()), int(t[1].item())
    tpot = np.nanmedian([m["tpot_s"] for m in mets]) * 1e3
    ttft = np.nanmedian([m["ttft_s"] for m in mets]) * 1e3
    e2e = np.nanmedian([m["e2e_s"] for m in mets]) * 1e3
    value = total / el
    if args.simulate_tp > 1:
        par = f"tp{args.simulate_tp}-simulated-" + (f"comm-model-{args.sim_comm}" if args.sim_comm else "no-comm")
    else:
        par = (f"dp{world}xtp1" if world > 1 else "tp1") if dp else f"tp{world}"
    out = {
        "metric": "output_tokens_per_sec",
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8-weights/bf16" if args.fp8 else "bf16",
        "data": "synthetic prompts, random-init weights",
        "p50_tpot_ms": round(float(tpot), 3),
        "p50_ttft_ms": round(float(ttft), 3),
        "p50_request_latency_ms": round(float(e2e), 3),
        "config": {"model": model_name, "global_batch": batch, "seq_len": args.prompt_len + args.gen_len,
                   "prompt_len": args.prompt_len, "gen_len": args.gen_len, "parallelism": par,
                   "sampling": "greedy" if args.greedy else "temperature=1.0,top_p=0.95,top_k=50",
                   "kv_cache": args.kv_dtype,
                   "engine_stats": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()},
                   **({"phase_ms": eng.phase_summary()} if eng.timer.enabled else {})},
    }
    del eng, model
    return out


if __name__ == "__main__":
    main()
