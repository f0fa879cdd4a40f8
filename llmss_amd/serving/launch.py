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
    return p


def build_driver(model_path: str, args):
    tp, rank, world = initialize_distributed()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dtype = args.dtype or ("bf16" if dev.type == "cuda" else "fp32")
    model = build_model(model_path, tp, dtype, dev, fp8=args.fp8)
    tok = load_tokenizer(model_path, model.cfg.vocab_size)
    eng = LLMEngine(model, max_num_seqs=args.max_num_seqs, max_batched_tokens=args.max_batched_tokens,
                    block_size=args.block_size, max_model_len=args.max_model_len, use_graphs=not args.no_graphs,
                    eos_token_id=getattr(tok, "eos_token_id", None))
    return EngineDriver(eng), tok, model
