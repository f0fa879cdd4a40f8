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
from typing import List, Optional

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
    """HF-style causal LM over the native decoder (reference ``GPTJForCausalLM.forward``,
    ``gptj_modeling.py:568-634``; ``GPTBigCodeForCausalLM.forward``, ``gpt_bigcode_modeling.py:851-915``).

    Each call is ONE engine step over the whole batch: rows without a cached prefix run the flash
    prefill kernel, rows continuing a cached prefix run the paged extend kernel (chunked-prefill
    attention), single new tokens run the decode kernel. ``attention_mask`` ([B, past + S], 1 =
    real token) drops padding from the computation (each row is its own variable-length sequence,
    so left padding neither takes attention nor shifts positions; logits at padded positions are
    0). ``position_ids`` ([B, S]) override the positions used for RoPE / learned position
    embeddings; by default a row's tokens take consecutive positions after its cached ones.
    """

    def __init__(self, config, weights, max_blocks: int = 4096, block_size: int = 16):
        cfg = config if isinstance(config, ModelConfig) else ModelConfig.from_hf_dict(config.to_dict())
        tp = getattr(weights, "tp", None) or TPGroup()
        w = load_hf_weights(cfg, weights.reader, tp.size, tp.rank, device=weights.device, dtype=weights.dtype)
        self.model = DecoderLM(cfg, w, tp)
        self.config = cfg
        self.block_size = block_size
        self.max_blocks = max_blocks
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
                 labels=None, attention_mask=None, position_ids=None, **kw):
        unsupported = [k for k in ("head_mask", "inputs_embeds", "token_type_ids", "encoder_hidden_states")
                       if kw.get(k) is not None]
        if unsupported:
            raise NotImplementedError(f"CausalLM: {unsupported} are not supported")
        return self.forward(input_ids, past_key_values, use_cache, labels, attention_mask, position_ids)

    @torch.no_grad()
    def forward(self, input_ids, past_key_values: Optional[PagedPast] = None, use_cache: bool = False, labels=None,
                attention_mask=None, position_ids=None):
        dev = self.model.device
        B, S = input_ids.shape
        bs = self.block_size
        past = past_key_values or PagedPast([0] * B, [[] for _ in range(B)])
        if attention_mask is not None:
            am = attention_mask.to("cpu").bool()
            if am.shape[0] != B or am.shape[1] < S:
                raise ValueError(f"attention_mask {tuple(am.shape)} does not cover input_ids {(B, S)}")
            keep = am[:, -S:]
        else:
            keep = torch.ones(B, S, dtype=torch.bool)
        ids_cpu = input_ids.to("cpu")
        pos_cpu = position_ids.to("cpu") if position_ids is not None else None
        rows = []  # (b, kept columns, start)
        for b in range(B):
            cols = torch.nonzero(keep[b]).flatten()
            rows.append((b, cols, past.lens[b]))
        # decodes (one new token after a cached prefix) first, then prompt rows / chunks
        dec = [r for r in rows if len(r[1]) == 1 and r[2] > 0]
        ext = [r for r in rows if len(r[1]) > 0 and not (len(r[1]) == 1 and r[2] > 0)]
        order = dec + ext
        out = torch.zeros(B, S, self.model.plan.vocab_padded, dtype=torch.float32, device=dev)
        if order:
            # the whole step's block need first: a failed allocation then leaves the pool untouched
            needs = [max(0, -(-(start + len(cols)) // bs) - len(past.blocks[b])) for b, cols, start in order]
            if sum(needs) > len(self._free):
                raise RuntimeError("CausalLM: KV pool exhausted")
            for (b, _, _), need in zip(order, needs):
                if need:
                    past.blocks[b].extend(self._alloc(need))
            tok, pos, slots, qlens, ctx, bt_rows = [], [], [], [], [], []
            for b, cols, start in order:
                n = len(cols)
                blocks = past.blocks[b]
                tok.append(ids_cpu[b, cols])
                pos.append(pos_cpu[b, cols] if pos_cpu is not None else torch.arange(start, start + n))
                slots += [blocks[p // bs] * bs + p % bs for p in range(start, start + n)]
                qlens.append(n)
                ctx.append(start + n)
                bt_rows.append(blocks)
            nd = len(dec)
            qt = torch.tensor(qlens)
            ends = qt.cumsum(0)
            cu = torch.zeros(len(ext) + 1, dtype=torch.int32)
            cu[1:] = (ends[nd:] - (ends[nd - 1] if nd else 0)).to(torch.int32)
            has_prefix = any(start > 0 for _, _, start in ext)
            maxb = max(len(r) for r in bt_rows)
            bt = torch.zeros(len(order), maxb, dtype=torch.int32)
            for i, r in enumerate(bt_rows):
                bt[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
            kind = "prefill" if nd == 0 and not has_prefix else "extend"
            inp = StepInput(kind, torch.cat(tok).long().to(dev), torch.cat(pos).long().to(dev),
                            torch.tensor(slots, dtype=torch.int64, device=dev), cu_seqlens=cu.to(dev),
                            max_seqlen=int(qt[nd:].max()) if ext else 0, block_tables=bt.to(dev),
                            ctx_lens=torch.tensor(ctx, dtype=torch.int32, device=dev), max_ctx=maxb * bs,
                            num_decode=nd, has_prefix=has_prefix)
            if kind == "extend" and not ext:  # decodes only
                inp = StepInput("decode", inp.input_ids, inp.positions, inp.slots, block_tables=inp.block_tables,
                                ctx_lens=inp.ctx_lens, max_ctx=inp.max_ctx)
            logits = self.model.logits(self.model.hidden_states(inp, self.kv)).float()
            r0 = 0
            for (b, cols, start), n in zip(order, qlens):
                out[b, cols.to(dev)] = logits[r0:r0 + n]
                past.lens[b] = start + n
                r0 += n
        out = out[..., : self.config.vocab_size]
        loss = None
        if labels is not None:
            from .. import ops

            loss = ops.cross_entropy(out, labels.to(out.device))
        if not use_cache:
            self.release(past)
            past = None
        return CausalLMOutput(out, past, loss)


class Weights:
    """Reference ``Weights(filenames, device, dtype, process_group, aliases)`` (``utils/weights.py:9-115``)
    over the native mmap safetensors reader: shard reads copy only this rank's rows / columns."""

    def __init__(self, filenames, device, dtype, process_group=None, aliases=None):
        from ..utils.checkpoint import CheckpointReader
        from .tp_layers import as_group_view

        self.filenames = list(filenames)
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        self.dtype = dtype
        self.reader = CheckpointReader(self.filenames, aliases=aliases)
        self.process_group = as_group_view(process_group if process_group is not None else TPGroup())
        self.tp = self.process_group.tp  # the TPGroup behind whatever group the caller passed

    def _cast(self, t: torch.Tensor) -> torch.Tensor:
        if t.dtype not in (torch.int32, torch.int64):  # reference :66-69: integers keep their dtype
            t = t.to(self.dtype)
        return t.to(self.device)

    def get_filename(self, tensor_name: str):
        name = self.reader.resolve(tensor_name)
        return self.reader.routing[name], name

    def get_shape(self, tensor_name: str):
        return self.reader.shape(tensor_name)

    def get_tensor(self, tensor_name: str) -> torch.Tensor:
        return self._cast(self.reader.get(tensor_name))

    def get_partial_sharded(self, tensor_name: str, dim: int) -> torch.Tensor:
        """Rows (dim 0) or columns (dim 1) [rank * n // ws, (rank + 1) * n // ws) of the tensor."""
        if dim not in (0, 1):
            raise NotImplementedError("sharding is implemented for dim 0 (rows) and dim 1 (columns)")
        ws, r = self.process_group.size(), self.process_group.rank()
        blk = self.get_shape(tensor_name)[dim] // ws
        t = self.reader.rows(tensor_name, r * blk, (r + 1) * blk) if dim == 0 else \
            self.reader.cols(tensor_name, r * blk, (r + 1) * blk)
        return self._cast(t)

    def get_sharded(self, tensor_name: str, dim: int) -> torch.Tensor:
        size = self.get_shape(tensor_name)[dim]
        ws = self.process_group.size()
        assert size % ws == 0, f"The chosen size {size} is not compatible with sharding on {ws} shards"
        return self.get_partial_sharded(tensor_name, dim)

    def get_multi_weights_col(self, prefixes: List[str], dim: int = 0, quantize=None) -> torch.Tensor:
        return torch.cat([self.get_sharded(f"{p}.weight", dim=0) for p in prefixes], dim=dim)

    def get_multi_weights_row(self, prefix: str, quantize=None) -> torch.Tensor:
        return self.get_sharded(f"{prefix}.weight", dim=1)


class _FamilyLM(CausalLM):
    """A :class:`CausalLM` bound to one checkpoint family: the reference's per-family class names
    (``custom_modeling/__init__.py:1-2``), rejecting a config of another ``model_type``."""

    model_type = ""

    def __init__(self, config, weights, max_blocks: int = 4096, block_size: int = 16):
        mt = config.model_type if isinstance(config, ModelConfig) else getattr(config, "model_type", None)
        if mt != self.model_type:
            raise ValueError(f"{type(self).__name__} takes model_type {self.model_type!r}, got {mt!r}")
        super().__init__(config, weights, max_blocks, block_size)


class GPTJForCausalLM(_FamilyLM):
    """Reference ``gptj_modeling.py:514`` (interleaved-pair rotary, parallel attention + MLP block)."""
    model_type = "gptj"


class GPTBigCodeForCausalLM(_FamilyLM):
    """Reference ``gpt_bigcode_modeling.py:786`` (multi-query attention, fused ``c_attn``)."""
    model_type = "gpt_bigcode"


class GPT2LMHeadModel(_FamilyLM):
    model_type = "gpt2"


class LlamaForCausalLM(_FamilyLM):
    model_type = "llama"


MODEL_REGISTRY = {c.model_type: c for c in (GPT2LMHeadModel, GPTJForCausalLM, GPTBigCodeForCausalLM,
                                            LlamaForCausalLM)}
