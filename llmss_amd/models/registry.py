"""Reference-compatible model API: ``MODEL_REGISTRY[config.model_type](config, weights)``.

Reference: ``custom_modeling/__init__.py:4-7`` (``gptj``, ``gpt_bigcode``) used as
``model = MODEL_REGISTRY[model_type](config, weights)`` then
``outputs = model(input_ids, past_key_values=..., use_cache=True)`` with ``outputs.logits``
``[B, S, V]`` and ``outputs.past_key_values`` (generate.py:67,104; consumer_server.py:60,125).

:class:`CausalLM` keeps that calling convention as a thin façade over the native paged-KV decoder:
``past_key_values`` is an opaque :class:`PagedPast` (block tables into a private KV pool), not a
tuple of ``torch.cat``-grown tensors. Rows of a batch must be unpadded (each row is its own
sequence); logits are returned for every input position like the reference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ..parallel.dist import TPGroup
from .config import ModelConfig
from .decoder import DecoderLM, StepInput
from .weights import load_hf_weights


@dataclass
class CausalLMOutput:
    logits: torch.Tensor
    past_key_values: Optional["PagedPast"] = None
    loss: Optional[torch.Tensor] = None


class PagedPast:
    def __init__(self, lens, blocks):
        self.lens = lens  # tokens cached per row
        self.blocks = blocks  # list of block-id lists per row


class CausalLM:
    def __init__(self, config, weights, max_blocks: int = 4096, block_size: int = 16):
        cfg = config if isinstance(config, ModelConfig) else ModelConfig.from_hf_dict(config.to_dict())
        tp = getattr(weights, "tp", None) or TPGroup()
        w = load_hf_weights(cfg, weights.reader, tp.size, tp.rank, device=weights.device, dtype=weights.dtype)
        self.model = DecoderLM(cfg, w, tp)
        self.config = cfg
        self.block_size = block_size
        self.kv = self.model.allocate_kv_cache(max_blocks, block_size)
        self._free = list(range(max_blocks - 1, -1, -1))

    def eval(self):
        return self

    def _alloc(self, n):
        if len(self._free) < n:
            raise RuntimeError("CausalLM: KV pool exhausted")
        return [self._free.pop() for _ in range(n)]

    def release(self, past: Optional[PagedPast]):
        if past is not None:
            for b in past.blocks:
                self._free.extend(b)
            past.blocks = [[] for _ in past.blocks]

    @torch.no_grad()
    def __call__(self, input_ids, past_key_values: Optional[PagedPast] = None, use_cache: bool = False,
                 labels=None, **_):
        return self.forward(input_ids, past_key_values, use_cache, labels)

    @torch.no_grad()
    def forward(self, input_ids, past_key_values: Optional[PagedPast] = None, use_cache: bool = False, labels=None):
        dev = self.model.device
        B, S = input_ids.shape
        bs = self.block_size
        past = past_key_values or PagedPast([0] * B, [[] for _ in range(B)])
        # every row is processed as a prefill chunk that attends to its cached prefix: run row by row
        # through the decoder (prefill for the first call, token-by-token decode afterwards)
        logits = []
        for b in range(B):
            start = past.lens[b]
            need = -(-(start + S) // bs) - len(past.blocks[b])
            if need > 0:
                past.blocks[b].extend(self._alloc(need))
            blocks = past.blocks[b]
            pos = torch.arange(start, start + S, device=dev)
            slots = torch.tensor([blocks[p // bs] * bs + p % bs for p in range(start, start + S)], device=dev)
            ids = input_ids[b].to(dev)
            if start == 0:
                inp = StepInput("prefill", ids, pos, slots,
                                cu_seqlens=torch.tensor([0, S], dtype=torch.int32, device=dev), max_seqlen=S)
                h = self.model.hidden_states(inp, self.kv)
                logits.append(self.model.logits(h))
            else:
                bt = torch.tensor([blocks], dtype=torch.int32, device=dev)
                rows = []
                for j in range(S):  # incremental tokens: one decode step each
                    inp = StepInput("decode", ids[j:j + 1], pos[j:j + 1], slots[j:j + 1], block_tables=bt,
                                    ctx_lens=torch.tensor([start + j + 1], dtype=torch.int32, device=dev),
                                    max_ctx=len(blocks) * bs)
                    rows.append(self.model.logits(self.model.hidden_states(inp, self.kv)))
                logits.append(torch.cat(rows, 0))
            past.lens[b] = start + S
        out = torch.stack(logits, 0)[..., : self.config.vocab_size].float()
        loss = None
        if labels is not None:
            from ..ops.reference import cross_entropy

            loss = cross_entropy(out, labels.to(out.device))
        if not use_cache:
            self.release(past)
            past = None
        return CausalLMOutput(out, past, loss)


@dataclass
class Weights:
    """Reference ``Weights(filenames, device, dtype, process_group)`` equivalent (weights.py:9-32)."""

    filenames: list
    device: torch.device
    dtype: torch.dtype
    process_group: Optional[TPGroup] = None

    def __post_init__(self):
        from ..utils.checkpoint import CheckpointReader

        self.reader = CheckpointReader(self.filenames)
        self.tp = self.process_group

    def get_tensor(self, name):
        return self.reader.get(name, self.dtype).to(self.device)


MODEL_REGISTRY = {"gpt2": CausalLM, "gptj": CausalLM, "gpt_bigcode": CausalLM, "llama": CausalLM}
