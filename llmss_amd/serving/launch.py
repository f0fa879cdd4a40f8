"""Shared bootstrap for the serving entry points: distributed init, model/engine/driver."""
from __future__ import annotations

import torch

from ..engine import LLMEngine, build_model
from ..parallel.dist import initialize_distributed
from ..utils.tokenizer import load_tokenizer
from .driver import EngineDriver


def add_engine_args(p):
    g = p.add_argument_group("engine")
    g.add_argument("--dtype", default=None, help="bf16 (GPU) | fp32 (CPU)")
    g.add_argument("--fp8", action="store_true", help="fp8-e4m3 weights")
    g.add_argument("--max_num_seqs", type=int, default=256)
    g.add_argument("--max_batched_tokens", type=int, default=8192)
    g.add_argument("--max_model_len", type=int, default=None)
    g.add_argument("--block_size", type=int, default=16)
    g.add_argument("--no_graphs", action="store_true")
    g.add_argument("--dp", type=int, default=1,
                   help="data-parallel replicas: with torchrun, world = dp x tp (each replica's leader serves "
                        "from the broker); in a single process, one TP=1 replica per GPU behind a Router")
    return p


def _engine(model_path, tp, dev, args, tok=None):
    dtype = args.dtype or ("bf16" if dev.type == "cuda" else "fp32")
    model = build_model(model_path, tp, dtype, dev, fp8=args.fp8)
    tok = tok or load_tokenizer(model_path, model.cfg.vocab_size)
    eng = LLMEngine(model, max_num_seqs=args.max_num_seqs, max_batched_tokens=args.max_batched_tokens,
                    block_size=args.block_size, max_model_len=args.max_model_len, use_graphs=not args.no_graphs,
                    eos_token_id=getattr(tok, "eos_token_id", None))
    return eng, tok, model


def build_driver(model_path: str, args):
    """(driver, tokenizer, model). ``driver`` is an EngineDriver (this rank's replica) or, for
    ``--dp N`` in a single process, a Router over N single-GPU replicas."""
    dp = getattr(args, "dp", 1) or 1
    tp, rank, world = initialize_distributed(dp=dp if world_size_env() > 1 else 1)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if dp > 1 and world == 1:  # in-process replicas, one per device
        from .router import Router

        n = torch.cuda.device_count() if dev.type == "cuda" else dp
        if dev.type == "cuda" and n < dp:
            raise SystemExit(f"--dp {dp} needs {dp} GPUs, found {n}")
        drivers, tok, model = [], None, None
        for i in range(dp):
            d = torch.device("cuda", i) if dev.type == "cuda" else dev
            if dev.type == "cuda":
                torch.cuda.set_device(d)
            eng, tok, m = _engine(model_path, None, d, args, tok)
            model = model or m
            drivers.append(EngineDriver(eng))
        if dev.type == "cuda":
            torch.cuda.set_device(0)
        return Router(drivers), tok, model
    eng, tok, model = _engine(model_path, tp, dev, args)
    return EngineDriver(eng), tok, model


def world_size_env() -> int:
    import os

    return int(os.environ.get("WORLD_SIZE", "1") or 1)
