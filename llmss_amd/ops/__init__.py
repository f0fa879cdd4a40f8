"""Op API used by the models. Routing is by tensor device only:

* CUDA (HIP) tensors -> the hand-written gfx950 kernels (``ops/hip.py`` -> ``llmss_amd._C``);
  a missing extension raises, it never falls back to PyTorch.
* CPU tensors -> the PyTorch definitions in ``ops/reference.py`` (CPU plumbing path / oracle).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref

__all__ = ["add_norm", "embed", "rope_cache", "attn_prefill", "attn_decode", "attn_extend", "linear", "sample", "quant_fp8_rows",
           "rope_tables", "glu_interleave", "glu_split", "cross_entropy"]

rope_tables = ref.rope_tables
glu_interleave = ref.glu_interleave
glu_split = ref.glu_split


def _hip():
    from . import hip
    return hip


def add_norm(x, weight, bias, eps, rms, residual=None, out=None, fp8_out=False):
    """``fp8_out`` (GPU): also emit the output's per-token fp8 twin for a W8A8 consumer (ops/hip.py)."""
    if x.is_cuda:
        return _hip().add_norm(x, weight, bias, eps, rms, residual, out=out, fp8_out=fp8_out)
    if x.dim() == 3:  # column-chunked [C, T, CW] -> [T, C * CW]
        x = x.permute(1, 0, 2).reshape(x.shape[1], -1)
    y, r = ref.add_norm(x, weight, bias, eps, rms, residual)
    if out is not None:
        out.copy_(y)
        y = out
    return y, r


def embed(ids, wte, positions=None, wpe=None):
    if wte.is_cuda:
        return _hip().embed(ids, wte, positions, wpe)
    return ref.embed(ids, wte, positions, wpe)


def rope_cache(qkv, positions, cos, sin, k_cache, v_cache, slots, nh, nkv, D, rot, style, do_rope=True):
    """Returns the (rotated) bf16 qkv tensor; ``qkv`` may be a GPU split-K PartialSum."""
    if qkv.is_cuda:
        return _hip().rope_cache(qkv, positions, cos, sin, k_cache, v_cache, slots, nh, nkv, D, rot, style, do_rope)
    ref.rope_cache(qkv, positions, cos, sin, k_cache, v_cache, slots, nh, nkv, D, rot, style, do_rope)
    return qkv


def _into(y, out):
    if out is not None:
        out.copy_(y)
        return out
    return y


def attn_prefill(qkv, cu_seqlens, max_seqlen, nh, nkv, D, scale, out=None):
    if qkv.is_cuda:
        return _hip().attn_prefill(qkv, cu_seqlens, max_seqlen, nh, nkv, D, scale, out=out)
    return _into(ref.attn_prefill(qkv, cu_seqlens, nh, nkv, D, scale), out)


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, nh, nkv, D, scale, max_ctx, splits=None, out=None):
    if q.is_cuda:
        return _hip().attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, nh, nkv, D, scale, max_ctx,
                                  splits=splits, out=out)
    return _into(ref.attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, nh, nkv, D, scale), out)


def attn_extend(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_qlen, nh, nkv, D, scale, out=None,
                fp8_out=False):
    """Chunked-prefill attention over the paged cache (the chunk's K/V already written). ``fp8_out``: the GPU
    kernel also writes the per-token fp8 twin for a W8A8 consumer (ops.hip.attn_extend); ignored on the CPU."""
    if q.is_cuda:
        return _hip().attn_extend(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_qlen, nh, nkv, D, scale,
                                  out=out, fp8_out=fp8_out)
    return _into(ref.attn_extend(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, nh, nkv, D, scale), out)


def linear(x, w, bias=None, act="none", glu=False, w_scale: Optional[torch.Tensor] = None, partial_ok=False):
    """partial_ok: on GPU the result may be a split-K PartialSum that only add_norm consumes."""
    if x.is_cuda:
        return _hip().linear(x, w, bias, act, glu, w_scale, partial_ok=partial_ok)
    return ref.linear(x, w, bias, act, glu, w_scale)


def sample(logits, temperature, top_k, top_p, seeds, vocab=None):
    if logits.is_cuda:
        return _hip().sample(logits, temperature, top_k, top_p, seeds, vocab)
    lg = logits if vocab is None else logits[:, :vocab]
    return ref.sample(lg, temperature, top_k, top_p, seeds)


def cross_entropy(logits, labels, ignore_index: int = -100):
    """Shifted LM loss (position t predicts label t+1), mean over non-ignored labels (reference
    gptj_modeling.py:612-622). GPU: the one-pass logsumexp kernel (csrc/loss.hip)."""
    if not logits.is_cuda:
        return ref.cross_entropy(logits, labels)
    V = logits.shape[-1]
    lab = torch.full(labels.shape, -1, dtype=torch.int64, device=logits.device)
    lab[..., :-1] = labels[..., 1:].to(logits.device)
    lab[lab == ignore_index] = -1
    # rows keep their (possibly vocab-padded) stride when the leading dims are uniformly strided
    lead = logits.shape[:-1]
    uniform = all(logits.stride(i) == logits.stride(i + 1) * logits.shape[i + 1] for i in range(logits.dim() - 2))
    rows = torch.as_strided(logits, (lead.numel(), V), (logits.stride(-2), 1)) if uniform and logits.stride(-1) == 1 \
        else logits.reshape(-1, V).contiguous()
    if rows.stride(0) % 8 or rows.data_ptr() % 16:  # the kernel's 16-B row loads: pad the row stride
        rows = torch.nn.functional.pad(rows, (0, (-V) % 8))
    loss = _hip().ce_loss_rows(rows, lab.reshape(-1), V)
    valid = (lab.reshape(-1) >= 0)
    return loss.sum() / valid.sum().clamp(min=1)


CAND_K = 64
CAND_KC = 128


def cand_ok(temperature, top_k) -> bool:
    """Rows the vocab-parallel candidate sampler reproduces exactly: greedy, or 1 <= top_k <= CAND_K."""
    import numpy as np

    t = np.asarray(temperature, dtype=np.float32)
    k = np.asarray(top_k, dtype=np.int64)
    return bool(np.all(~(t > 0) | (k == 1) | ((k >= 1) & (k <= CAND_K))))


def sample_distributed(local, tp, lo, V, temperature, top_k, top_p, seeds, out=None, shards=1):
    """Vocab-parallel sampling without gathering logits: per-rank candidates -> all-gather -> select.
    ``local`` = this rank's [B, V/tp] logit shard whose first column is global token ``lo``; ``shards`` > 1
    additionally cuts it into column shards inside one launch (a single GPU's full vocabulary)."""
    if local.is_cuda:
        h = _hip()
        pack = h.cand_topk(local, lo, V, temperature, top_k, shards=shards)
        allp = tp.all_gather_last_dim(pack)
        return h.sample_cand(allp, h.CAND_KC, temperature, top_k, top_p, seeds, out=out)
    pack = ref.cand_topk(local, lo, V, temperature, top_k, CAND_K, CAND_KC)
    allp = tp.all_gather_last_dim(pack)
    y = ref.sample_cand(allp, allp.shape[1] // (2 * CAND_KC), CAND_KC, temperature, top_k, top_p, seeds, V)
    return _into(y, out)


def quant_fp8_rows(w):
    if w.is_cuda:
        return _hip().quant_fp8_rows(w)
    return ref.quant_fp8_rows(w)
