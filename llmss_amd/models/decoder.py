"""Family-agnostic tensor-parallel decoder forward over a paged KV cache.

Replaces the per-family modeling files of the reference (``gptj_modeling.py`` 648 lines,
``gpt_bigcode_modeling.py`` 926 lines, HF ``PreTrainedModel`` glue) with one forward that
covers GPT-2, GPT-J (parallel block), GPT-BigCode (MQA/MHA) and Llama (RMSNorm/SwiGLU/GQA):

    per layer (sequential):  y = norm1(x + delta)          fused residual add + norm (K3/K17)
                             qkv = y @ Wqkv (+b)            column-parallel GEMM (K4)
                             rope + paged KV write          in place (K8/K10)
                             a = attention(q, cache)        prefill flash / split-K decode (K11-14)
                             o = a @ Wo (+b rank 0)         row-parallel GEMM (K6) -> all-reduce
                             y2 = norm2(x + o)
                             m = act(y2 @ Wup (+b))         GEMM with fused GELU / SwiGLU epilogue
                             delta = m @ Wdown -> all-reduce
    GPT-J (parallel):        delta = (a @ Wo) + mlp(y) -> ONE all-reduce per layer (the reference
                             all-reduces twice per layer)

Tokens of all sequences in a step are flattened ([T, H]); the LM head runs on the last token of
each sequence only (the reference runs it on every prompt position, K7) and is vocab-parallel
followed by an all-gather of [B, V/tp] logits.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from .. import ops
from ..parallel.dist import TPGroup
from .config import ModelConfig
from .weights import ModelWeights, ShardPlan, shard_plan


def _hip_ops():
    from ..ops import hip

    return hip


@dataclass
class StepInput:
    kind: str  # "prefill" | "decode"
    input_ids: torch.Tensor  # [T] int64
    positions: torch.Tensor  # [T] int64
    slots: torch.Tensor  # [T] int64 physical KV slots (-1 = do not cache)
    cu_seqlens: Optional[torch.Tensor] = None  # prefill: [B+1] int32
    max_seqlen: int = 0
    block_tables: Optional[torch.Tensor] = None  # decode: [B, maxb] int32
    ctx_lens: Optional[torch.Tensor] = None  # decode: [B] int32
    max_ctx: int = 0
    decode_splits: Optional[Tuple[int, int]] = None
    last_idx: Optional[torch.Tensor] = None  # rows feeding the LM head ([B] int64); None = all rows


class DecoderLM:
    def __init__(self, cfg: ModelConfig, weights: ModelWeights, tp: Optional[TPGroup] = None):
        self.cfg = cfg
        self.w = weights
        self.tp = tp or TPGroup()
        self.plan: ShardPlan = shard_plan(cfg, self.tp.size, self.tp.rank)
        self.scale = cfg.head_dim ** -0.5
        self.rms = cfg.norm == "rmsnorm"
        self.act = "none" if cfg.gated_mlp else cfg.activation
        # TP all-reduce / GEMM overlap for large steps (prefill): row chunks of this many tokens
        self.overlap_rows = int(os.environ.get("LLMSS_TP_OVERLAP_ROWS", "4096"))
        # fused RoPE+KV-write+attention decode: correct, but measured slower (its prologue halves the
        # attention kernel's occupancy), so opt-in
        self.fused_decode = os.environ.get("LLMSS_FUSED_DECODE", "0") == "1"
        self._comm_stream = None

    @property
    def device(self):
        return self.w.wte.device

    @property
    def dtype(self):
        return self.w.wte.dtype

    # --------------------------------------------------------------------------------- KV
    def kv_cache_shape(self, num_blocks: int, block_size: int):
        return (num_blocks, self.plan.nkv_l, block_size, self.cfg.head_dim)

    def kv_bytes_per_block(self, block_size: int) -> int:
        return 2 * self.cfg.num_layers * self.plan.nkv_l * block_size * self.cfg.head_dim * 2

    def allocate_kv_cache(self, num_blocks: int, block_size: int):
        shp = self.kv_cache_shape(num_blocks, block_size)
        return [(torch.zeros(shp, dtype=self.dtype, device=self.device),
                 torch.zeros(shp, dtype=self.dtype, device=self.device)) for _ in range(self.cfg.num_layers)]

    # ---------------------------------------------------------------------------- forward
    def _attention(self, qkv, inp: StepInput, kc, vc):
        cfg, p = self.cfg, self.plan
        D = cfg.head_dim
        do_rope = cfg.position == "rope"
        if inp.kind == "decode" and qkv.is_cuda and self.fused_decode and \
                _hip_ops().fused_decode_ok(D, cfg.rotary_dim, cfg.rope_style, do_rope):
            # one launch: RoPE + paged KV write of the new token + attention (no rope_cache kernel)
            return _hip_ops().attn_decode_fused(
                qkv, inp.positions, self.w.cos, self.w.sin, kc, vc, inp.slots, inp.block_tables, inp.ctx_lens,
                p.nh_l, p.nkv_l, D, cfg.rotary_dim, cfg.rope_style, self.scale, inp.max_ctx, do_rope=do_rope,
                splits=inp.decode_splits)
        qkv = ops.rope_cache(qkv, inp.positions, self.w.cos, self.w.sin, kc, vc, inp.slots, p.nh_l, p.nkv_l, D,
                             cfg.rotary_dim, cfg.rope_style, do_rope=cfg.position == "rope")
        if inp.kind == "prefill":
            return ops.attn_prefill(qkv, inp.cu_seqlens, inp.max_seqlen, p.nh_l, p.nkv_l, D, self.scale)
        return ops.attn_decode(qkv, kc, vc, inp.block_tables, inp.ctx_lens, p.nh_l, p.nkv_l, D, self.scale,
                               inp.max_ctx, splits=inp.decode_splits)

    def _reduce_rows(self, fn, *inputs) -> torch.Tensor:
        """``all_reduce(fn(*inputs))`` for a row-parallel projection (or a whole MLP).

        Large steps run in row chunks: chunk c's RCCL all-reduce is issued on a high-priority comm
        stream while the compute stream already runs chunk c+1's GEMMs, so the per-layer
        all-reduce hides behind the next GEMM (prefill at TP=8 moves ~0.5 GB per all-reduce). Decode
        steps (a few MB, latency-bound) keep one all-reduce.
        """
        if not self.tp.is_real:
            return fn(*inputs)
        M = inputs[0].shape[0]
        step = self.overlap_rows
        if M <= step or step <= 0:
            return self.tp.all_reduce(fn(*inputs))
        if not inputs[0].is_cuda:  # gloo / CPU: same chunking (numerics), no streams
            return torch.cat([self.tp.all_reduce(fn(*(t[r:r + step] for t in inputs))) for r in range(0, M, step)])
        cur = torch.cuda.current_stream()
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(device=inputs[0].device, priority=-1)
        comm = self._comm_stream
        outs = []
        for r in range(0, M, step):
            y = fn(*(t[r:r + step] for t in inputs))
            comm.wait_stream(cur)  # chunk r's GEMM done
            with torch.cuda.stream(comm):
                self.tp.all_reduce(y)
            y.record_stream(comm)
            outs.append(y)
        cur.wait_stream(comm)
        return torch.cat(outs)

    def hidden_states(self, inp: StepInput, kv_caches) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        eps, rms = cfg.norm_eps, self.rms
        x = ops.embed(inp.input_ids, w.wte, inp.positions if w.wpe is not None else None, w.wpe)
        residual = None
        delta = x
        fuse = self.tp.size == 1  # split-K partials can skip their own reduce only without a TP all-reduce
        for i, L in enumerate(w.layers):
            kc, vc = kv_caches[i]
            y, residual = ops.add_norm(delta, L.ln1_w, L.ln1_b, eps, rms, residual)
            # column-parallel QKV: its split-K partials are summed inside the rope/cache kernel
            a = self._attention(L.qkv(y, partial_ok=True), inp, kc, vc)
            if cfg.parallel_block:  # GPT-J: one all-reduce for attention + MLP
                delta = self._reduce_rows(lambda a_, y_: L.o(a_).add_(L.down(L.up(y_, self.act))), a, y)
            elif fuse:
                # TP=1: the split-K partials of o / down are reduced inside the next add_norm
                o = L.o(a, partial_ok=True)
                y2, residual = ops.add_norm(o, L.ln2_w, L.ln2_b, eps, rms, residual)
                delta = L.down(L.up(y2, self.act), partial_ok=True)
            else:
                o = self._reduce_rows(L.o, a)
                y2, residual = ops.add_norm(o, L.ln2_w, L.ln2_b, eps, rms, residual)
                delta = self._reduce_rows(lambda y_: L.down(L.up(y_, self.act)), y2)
        h, _ = ops.add_norm(delta, w.lnf_w, w.lnf_b, eps, rms, residual)
        return h

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """[B, H] -> full-vocab logits [B, Vpadded] (all-gathered across TP ranks)."""
        local = self.w.head(h)
        return self.tp.all_gather_last_dim(local)

    def forward(self, inp: StepInput, kv_caches) -> torch.Tensor:
        h = self.hidden_states(inp, kv_caches)
        if inp.last_idx is not None:
            h = h.index_select(0, inp.last_idx)
        return self.logits(h)

    __call__ = forward
