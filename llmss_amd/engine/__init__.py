"""Engine construction helpers shared by generate.py, the servers and bench.py."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..models.config import ModelConfig, get_preset
from ..models.decoder import DecoderLM
from ..models.weights import load_hf_weights, load_shard, random_weights, save_shard, shard_cache_path
from ..parallel.dist import TPGroup
from ..utils.checkpoint import CheckpointReader, weight_files
from .engine import LLMEngine, Request, StepEvent
from .sampling import SamplingParams

__all__ = ["LLMEngine", "SamplingParams", "Request", "StepEvent", "build_model", "build_engine"]

_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32}


def default_device(tp: TPGroup) -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def build_model(model: str, tp: Optional[TPGroup] = None, dtype: str = "bf16", device=None, fp8: bool = False,
                random_init: Optional[bool] = None, seed: int = 0, shard_cache: Optional[str] = None) -> DecoderLM:
    """``model`` is a HF checkpoint directory or a preset name (random-init weights).

    ``shard_cache`` (or ``LLMSS_SHARD_CACHE``): directory of finished per-rank weight shards; the
    first load writes this rank's file, later loads mmap it instead of re-sharding the checkpoint.
    """
    tp = tp or TPGroup()
    device = torch.device(device) if device is not None else default_device(tp)
    if device.type == "cuda":
        if dtype not in ("bf16", "bfloat16"):
            raise ValueError("the gfx950 kernels compute in bf16 (optionally fp8 weights)")
    tdtype = _DTYPES[dtype]
    is_dir = os.path.isdir(model)
    if random_init is None:
        random_init = not is_dir
    if is_dir:
        cfg = ModelConfig.from_pretrained(model)
    else:
        cfg = get_preset(model)
    if random_init:
        w = random_weights(cfg, tp.size, tp.rank, device=device, dtype=tdtype, seed=seed, fp8=fp8)
    else:
        files = weight_files(model)
        shard_cache = shard_cache or os.environ.get("LLMSS_SHARD_CACHE")
        cpath = shard_cache_path(shard_cache, model, files, tp.size, tp.rank, tdtype, fp8) if shard_cache else None
        if cpath and os.path.exists(cpath):
            w = load_shard(cfg, cpath, device, tdtype)
        else:
            w = load_hf_weights(cfg, CheckpointReader(files), tp.size, tp.rank, device=device, dtype=tdtype, fp8=fp8)
            if cpath:
                save_shard(w, cpath)
    return DecoderLM(cfg, w, tp)


def build_engine(model: str, tp: Optional[TPGroup] = None, dtype: str = "bf16", device=None, fp8: bool = False,
                 random_init: Optional[bool] = None, **engine_kw) -> LLMEngine:
    m = build_model(model, tp, dtype, device, fp8, random_init)
    return LLMEngine(m, **engine_kw)
