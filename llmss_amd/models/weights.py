"""Canonical rank-local weight layout, tensor-parallel sharding and loading.

One layout serves every family (the decoder in ``decoder.py`` is family-agnostic):

* ``qkv_w``  [nh_l*D + 2*nkv_l*D, H]  column-parallel, q|k|v fused at load time
  (reference loads separate q/k/v for GPT-J, ``gptj_modeling.py:84-92``, and for BigCode loads
  the FULL c_attn on every rank then slices, ``gpt_bigcode_modeling.py:122-155`` - quirk Q8).
* ``o_w``    [H, nh_l*D]  row-parallel; its bias lives on rank 0 only (``layers.py:161-173``).
* ``up_w``   [F_l, H] or, for SwiGLU, [2*F_l, H] with gate/up interleaved in 16-row groups so
  the GEMM epilogue emits silu(gate)*up directly.
* ``down_w`` [H, F_l] row-parallel (bias on rank 0).
* ``wte``    full table replicated on every rank (no embedding all-reduce; reference C1).
* ``head_w`` [Vp/tp, H] vocab-parallel with the vocab padded to a multiple of 16*tp (fixes the
  reference's silent loss of ids >= tp*floor(V/tp), quirk Q6); GPT-J's lm_head bias is loaded
  (the reference drops it, quirk Q5). Tied heads (GPT-2, BigCode) share the checkpoint tensor
  (read once per rank; the reference loads wte twice, Q9).

KV heads: sharded when nkv >= tp, otherwise each rank keeps exactly the kv head(s) its query
heads use (MQA: every rank holds the single kv head), generalising the reference's MQA
replication (``gpt_bigcode_modeling.py:150-155``) to GQA.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .. import ops
from ..ops import reference as ref
from .config import ModelConfig


@dataclass
class ShardPlan:
    tp: int
    rank: int
    nh_l: int
    kv_start: int
    nkv_l: int
    F_l: int
    vocab_padded: int

    @property
    def v_l(self) -> int:
        return self.vocab_padded // self.tp


# load neox-RoPE checkpoints with q / k head dims interleaved (gptj-form rotation, fusable into the QKV epilogue)
ROPE_INTERLEAVE = True

def shard_plan(cfg: ModelConfig, tp: int, rank: int) -> ShardPlan:
    nh, nkv = cfg.num_heads, cfg.num_kv_heads
    if nh % tp:
        raise ValueError(f"{cfg.model_type}: num_heads={nh} is not divisible by tp={tp}")
    nh_l = nh // tp
    G = nh // nkv
    kv_start = (rank * nh_l) // G
    kv_end = ((rank + 1) * nh_l - 1) // G + 1
    nkv_l = kv_end - kv_start
    if nh_l % nkv_l or (nh_l // nkv_l) != min(G, nh_l):
        raise ValueError(f"cannot shard {nh} q heads / {nkv} kv heads over tp={tp}")
    if cfg.intermediate_size % tp:
        raise ValueError(f"intermediate_size {cfg.intermediate_size} not divisible by tp={tp}")
    F_l = cfg.intermediate_size // tp
    if cfg.gated_mlp and F_l % 16:
        raise ValueError("gated MLP width per rank must be a multiple of 16")
    vp = math.ceil(cfg.vocab_size / (16 * tp)) * 16 * tp
    return ShardPlan(tp, rank, nh_l, kv_start, nkv_l, F_l, vp)


@dataclass
class Linear:
    # [N, K] bf16, or uint8 fp8-e4m3 when w_scale is set (per-row scales)
    w: torch.Tensor
    b: Optional[torch.Tensor] = None
    w_scale: Optional[torch.Tensor] = None
    glu: bool = False

    def __call__(self, x, act="none", partial_ok=False):
        return ops.linear(x, self.w, self.b, act, self.glu, self.w_scale, partial_ok=partial_ok)

    @property
    def N(self) -> int:
        return self.w.shape[0]

    @property
    def K(self) -> int:
        return self.w.shape[1]

    def rows(self, r0: int, r1: int) -> "Linear":
        """Output features [r0, r1) as a Linear over views (no copy): the weight slice a column chunk of a
        row-parallel projection reads (DecoderLM._reduce_cols)."""
        if self.glu:
            raise ValueError("row slices of SwiGLU linears are not supported")
        return Linear(self.w[r0:r1], None if self.b is None else self.b[r0:r1],
                      None if self.w_scale is None else self.w_scale[r0:r1], False)

    def dense(self) -> torch.Tensor:
        """The [N, K] row-major weight."""
        return self.w

    @property
    def out_features(self):
        return self.N // (2 if self.glu else 1)


@dataclass
class LayerWeights:
    ln1_w: torch.Tensor
    ln1_b: Optional[torch.Tensor]
    ln2_w: Optional[torch.Tensor]
    ln2_b: Optional[torch.Tensor]
    qkv: Linear
    o: Linear
    up: Linear
    down: Linear


@dataclass
class ModelWeights:
    wte: torch.Tensor
    wpe: Optional[torch.Tensor]
    layers: List[LayerWeights]
    lnf_w: torch.Tensor
    lnf_b: Optional[torch.Tensor]
    head: Linear
    cos: Optional[torch.Tensor] = None
    sin: Optional[torch.Tensor] = None
    extra: dict = field(default_factory=dict)
    # neox RoPE models: q / k head dims were interleaved at load (ref.rope_interleave_rows), so the
    # model applies gptj-style RoPE to them (DecoderLM.rope_style)
    rope_interleaved: bool = False

    def nbytes(self) -> int:
        """Device bytes held (views sharing one allocation, like a tied embedding / head, count once)."""
        seen, tot = set(), 0
        for t in _tensors(self):
            st = t.untyped_storage()
            if st.data_ptr() not in seen:
                seen.add(st.data_ptr())
                tot += st.nbytes()
        return tot


def _tensors(mw: ModelWeights):
    yield mw.wte
    if mw.wpe is not None:
        yield mw.wpe
    for L in mw.layers:
        for t in (L.ln1_w, L.ln1_b, L.ln2_w, L.ln2_b):
            if t is not None:
                yield t
        for lin in (L.qkv, L.o, L.up, L.down):
            yield lin.w
            if lin.b is not None:
                yield lin.b
    yield mw.lnf_w
    yield mw.head.w


# ------------------------------------------------------------------------------ finalisation
def _finish(cfg: ModelConfig, plan: ShardPlan, wte, wpe, layers_raw, lnf_w, lnf_b, head_w, head_b, device, dtype,
            fp8: bool) -> ModelWeights:
    """Move to device / dtype, pad the head vocab, interleave SwiGLU, optional fp8 quant."""

    def dev(t):
        if t is None:
            return None
        return t.to(device=device, dtype=dtype if t.is_floating_point() else t.dtype).contiguous()

    def lin(w, b, glu=False, quant=False):
        w = dev(w)
        b = dev(b)
        if quant and fp8:
            q, s = ops.quant_fp8_rows(w)
            return Linear(q, b, s, glu)
        return Linear(w, b, None, glu)

    # neox RoPE: interleave the q / k head dims (ROPE_INTERLEAVE = False keeps the checkpoint order; tests)
    il = cfg.position == "rope" and cfg.rope_style == "neox" and ROPE_INTERLEAVE
    layers = []
    for d in layers_raw:
        if il:
            d = dict(d)
            d["qkv_w"] = ref.rope_interleave_rows(d["qkv_w"], plan.nh_l, plan.nkv_l, cfg.head_dim, cfg.rotary_dim)
            if d.get("qkv_b") is not None:
                d["qkv_b"] = ref.rope_interleave_rows(d["qkv_b"], plan.nh_l, plan.nkv_l, cfg.head_dim,
                                                      cfg.rotary_dim)
        if cfg.gated_mlp:
            up_w = ref.glu_interleave(d["gate_w"], d["up_w"], 0)
            up_b = ref.glu_interleave(d["gate_b"], d["up_b"], 0) if d.get("gate_b") is not None else None
        else:
            up_w, up_b = d["up_w"], d.get("up_b")
        layers.append(LayerWeights(
            ln1_w=dev(d["ln1_w"]), ln1_b=dev(d.get("ln1_b")), ln2_w=dev(d.get("ln2_w")), ln2_b=dev(d.get("ln2_b")),
            qkv=lin(d["qkv_w"], d.get("qkv_b"), quant=True), o=lin(d["o_w"], d.get("o_b"), quant=True),
            up=lin(up_w, up_b, glu=cfg.gated_mlp, quant=True), down=lin(d["down_w"], d.get("down_b"), quant=True),
        ))
    # vocab-parallel head with padding
    vl = plan.v_l
    lo = plan.rank * vl
    n = max(0, min(cfg.vocab_size, lo + vl) - lo)
    hb = None
    if head_b is not None:
        hb = torch.zeros(vl, dtype=head_b.dtype, device=head_b.device)
        if n:
            hb[:n] = head_b[lo:lo + n]
    if head_w is wte:
        # tied embedding / head (GPT-2, BigCode): ONE device table [Vpadded, H]; the embedding is its
        # first V rows and this rank's head shard is rows [lo, lo + vl) of it - no second copy in HBM
        # (the reference loads the tied table twice, gpt_bigcode_modeling.py:564,793-797)
        table = torch.zeros(plan.vocab_padded, cfg.hidden_size, dtype=dtype, device=device)
        table[:cfg.vocab_size].copy_(wte.to(device=device, dtype=dtype))
        wte_d, head = table[:cfg.vocab_size], Linear(table[lo:lo + vl], dev(hb))
    else:
        hw = torch.zeros(vl, cfg.hidden_size, dtype=head_w.dtype, device=head_w.device)
        if n:
            hw[:n] = head_w[lo:lo + n]
        wte_d, head = dev(wte), lin(hw, hb)
    mw = ModelWeights(wte=wte_d, wpe=dev(wpe), layers=layers, lnf_w=dev(lnf_w), lnf_b=dev(lnf_b), head=head,
                      rope_interleaved=il)
    if cfg.position == "rope":
        cos, sin = ref.rope_tables(cfg.max_position_embeddings, cfg.rotary_dim, cfg.rope_theta, device)
        mw.cos, mw.sin = cos, sin
    return mw


# ------------------------------------------------------------------------------ random init
def random_weights(cfg: ModelConfig, tp: int = 1, rank: int = 0, device="cpu", dtype=torch.bfloat16,
                   seed: int = 0, std: float = 0.02, fp8: bool = False) -> ModelWeights:
    """Random-init rank-local weights of the architecture (synthetic benches/tests).

    Tensors are generated directly at their rank-local shapes on ``device`` (no full-model
    materialisation). Norm weights are 1, biases small.
    """
    plan = shard_plan(cfg, tp, rank)
    H, D = cfg.hidden_size, cfg.head_dim
    gen_dev = torch.device(device)
    g = torch.Generator(device=gen_dev)
    g.manual_seed(seed * 1000 + rank)
    # replicated tensors (embeddings, norm biases, rank-0 row-parallel biases, the final norm) come
    # from a rank-independent stream: every rank must hold the same copy, as after a checkpoint load
    g_rep = torch.Generator(device=gen_dev)
    g_rep.manual_seed(seed * 1000 + 999)

    def rn(*shape, s=std, rep=False):
        return (torch.randn(*shape, generator=g_rep if rep else g, device=gen_dev, dtype=torch.float32) * s).to(dtype)

    def ones(n):
        return torch.ones(n, device=gen_dev, dtype=dtype)

    layers = []
    qkv_n = (plan.nh_l + 2 * plan.nkv_l) * D
    for _ in range(cfg.num_layers):
        d = dict(
            ln1_w=ones(H), ln1_b=rn(H, rep=True) if cfg.norm == "layernorm" else None,
            qkv_w=rn(qkv_n, H), qkv_b=rn(qkv_n) if cfg.qkv_bias else None,
            o_w=rn(H, plan.nh_l * D, s=std / math.sqrt(2 * cfg.num_layers)),
            o_b=rn(H, rep=True) if cfg.out_bias else None,
            down_w=rn(H, plan.F_l, s=std / math.sqrt(2 * cfg.num_layers)),
            down_b=rn(H, rep=True) if cfg.mlp_bias else None,
        )
        if rank != 0:  # drawn on every rank (keeps the replicated stream aligned), kept on rank 0 only
            d["o_b"] = d["down_b"] = None
        if not cfg.parallel_block:
            d["ln2_w"], d["ln2_b"] = ones(H), (rn(H, rep=True) if cfg.norm == "layernorm" else None)
        if cfg.gated_mlp:
            d["gate_w"], d["up_w"] = rn(plan.F_l, H), rn(plan.F_l, H)
            if cfg.mlp_bias:
                d["gate_b"], d["up_b"] = rn(plan.F_l), rn(plan.F_l)
        else:
            d["up_w"] = rn(plan.F_l, H)
            d["up_b"] = rn(plan.F_l) if cfg.mlp_bias else None
        layers.append(d)
    wte = rn(cfg.vocab_size, H, rep=True)
    wpe = rn(cfg.max_position_embeddings, H, s=0.01, rep=True) if cfg.position == "learned" else None
    if cfg.tie_word_embeddings:
        head_w_full = wte
    else:
        head_w_full = None
    # head shard generated directly (untied) to avoid a full [V, H] second table
    vl = plan.v_l
    lo = rank * vl
    n = max(0, min(cfg.vocab_size, lo + vl) - lo)
    if head_w_full is None:
        head_w = torch.zeros(plan.vocab_padded, H, dtype=dtype, device=gen_dev)
        if n:
            head_w[lo:lo + n] = rn(n, H)
    else:
        head_w = head_w_full
    head_b = None
    if cfg.lm_head_bias:
        head_b = torch.zeros(plan.vocab_padded, dtype=dtype, device=gen_dev)
        if n:
            head_b[lo:lo + n] = rn(n)
    lnf_b = rn(H, rep=True) if cfg.norm == "layernorm" else None
    return _finish(cfg, plan, wte, wpe, layers, ones(H), lnf_b, head_w, head_b, device, dtype, fp8)


# ------------------------------------------------------------------------------ HF checkpoints
def _prefix(reader, *cands):
    for c in cands:
        if any(k.startswith(c) for k in reader.keys()):
            return c
    return ""


def load_hf_weights(cfg: ModelConfig, reader, tp: int = 1, rank: int = 0, device="cpu",
                    dtype=torch.bfloat16, fp8: bool = False) -> ModelWeights:
    """Read a HF checkpoint's tensors for this rank only (sharded reads) and finalise."""
    plan = shard_plan(cfg, tp, rank)
    H, D = cfg.hidden_size, cfg.head_dim
    nh_l, nkv_l = plan.nh_l, plan.nkv_l
    q0, q1 = rank * nh_l * D, (rank + 1) * nh_l * D
    k0, k1 = plan.kv_start * D, (plan.kv_start + nkv_l) * D
    f0, f1 = rank * plan.F_l, (rank + 1) * plan.F_l
    fdt = torch.float32  # read in checkpoint precision, cast once on device
    mt = cfg.model_type
    layers = []

    if mt == "gpt2":
        p = _prefix(reader, "transformer.h.", "h.")
        p = p[:-2] if p else ""
        top = "transformer." if p.startswith("transformer") else ""
        for i in range(cfg.num_layers):
            b = f"{p}h.{i}."
            ca = b + "attn.c_attn."  # Conv1D [H, 3H]
            qkv_w = torch.cat([reader.cols(ca + "weight", q0, q1, fdt), reader.cols(ca + "weight", H + k0, H + k1, fdt),
                               reader.cols(ca + "weight", 2 * H + k0, 2 * H + k1, fdt)], 1).t()
            cb = reader.get(ca + "bias", fdt)
            qkv_b = torch.cat([cb[q0:q1], cb[H + k0:H + k1], cb[2 * H + k0:2 * H + k1]])
            layers.append(dict(
                ln1_w=reader.get(b + "ln_1.weight"), ln1_b=reader.get(b + "ln_1.bias"),
                ln2_w=reader.get(b + "ln_2.weight"), ln2_b=reader.get(b + "ln_2.bias"),
                qkv_w=qkv_w, qkv_b=qkv_b,
                o_w=reader.rows(b + "attn.c_proj.weight", q0, q1, fdt).t(),
                o_b=reader.get(b + "attn.c_proj.bias") if rank == 0 else None,
                up_w=reader.cols(b + "mlp.c_fc.weight", f0, f1, fdt).t(),
                up_b=reader.get(b + "mlp.c_fc.bias", fdt)[f0:f1],
                down_w=reader.rows(b + "mlp.c_proj.weight", f0, f1, fdt).t(),
                down_b=reader.get(b + "mlp.c_proj.bias") if rank == 0 else None,
            ))
        wte = reader.get(top + "wte.weight")
        wpe = reader.get(top + "wpe.weight")
        lnf_w, lnf_b = reader.get(top + "ln_f.weight"), reader.get(top + "ln_f.bias")
        head_w = reader.get("lm_head.weight") if (not cfg.tie_word_embeddings and reader.has("lm_head.weight")) else wte
        head_b = None
    elif mt == "gptj":
        for i in range(cfg.num_layers):
            b = f"transformer.h.{i}."
            a = b + "attn."
            qkv_w = torch.cat([reader.rows(a + "q_proj.weight", q0, q1, fdt), reader.rows(a + "k_proj.weight", k0, k1, fdt),
                               reader.rows(a + "v_proj.weight", k0, k1, fdt)], 0)
            layers.append(dict(
                ln1_w=reader.get(b + "ln_1.weight"), ln1_b=reader.get(b + "ln_1.bias"),
                qkv_w=qkv_w, o_w=reader.cols(a + "out_proj.weight", q0, q1, fdt),
                up_w=reader.rows(b + "mlp.fc_in.weight", f0, f1, fdt), up_b=reader.get(b + "mlp.fc_in.bias")[f0:f1],
                down_w=reader.cols(b + "mlp.fc_out.weight", f0, f1, fdt),
                down_b=reader.get(b + "mlp.fc_out.bias") if rank == 0 else None,
            ))
        wte = reader.get("transformer.wte.weight")
        wpe = None
        lnf_w, lnf_b = reader.get("transformer.ln_f.weight"), reader.get("transformer.ln_f.bias")
        head_w = reader.get("lm_head.weight")
        head_b = reader.get("lm_head.bias") if reader.has("lm_head.bias") else None
    elif mt == "gpt_bigcode":
        nkv = cfg.num_kv_heads
        for i in range(cfg.num_layers):
            b = f"transformer.h.{i}."
            ca = b + "attn.c_attn."
            if nkv == cfg.num_heads:
                # MHA: nn.Linear [3H, H] laid out per head as [q_h | k_h | v_h] (HF view(nh, 3D))
                h0, h1 = rank * nh_l, (rank + 1) * nh_l
                blk = reader.rows(ca + "weight", 3 * D * h0, 3 * D * h1, fdt).view(nh_l, 3, D, H)
                qkv_w = torch.cat([blk[:, 0].reshape(-1, H), blk[:, 1].reshape(-1, H), blk[:, 2].reshape(-1, H)], 0)
                bb = reader.get(ca + "bias", fdt)[3 * D * h0:3 * D * h1].view(nh_l, 3, D)
                qkv_b = torch.cat([bb[:, 0].reshape(-1), bb[:, 1].reshape(-1), bb[:, 2].reshape(-1)])
            else:
                # MQA/GQA: nn.Linear [H + 2*nkv*D, H] = [q | k | v]
                kb, vb = H, H + nkv * D
                qkv_w = torch.cat([reader.rows(ca + "weight", q0, q1, fdt),
                                   reader.rows(ca + "weight", kb + k0, kb + k1, fdt),
                                   reader.rows(ca + "weight", vb + k0, vb + k1, fdt)], 0)
                cb = reader.get(ca + "bias", fdt)
                qkv_b = torch.cat([cb[q0:q1], cb[kb + k0:kb + k1], cb[vb + k0:vb + k1]])
            layers.append(dict(
                ln1_w=reader.get(b + "ln_1.weight"), ln1_b=reader.get(b + "ln_1.bias"),
                ln2_w=reader.get(b + "ln_2.weight"), ln2_b=reader.get(b + "ln_2.bias"),
                qkv_w=qkv_w, qkv_b=qkv_b,
                o_w=reader.cols(b + "attn.c_proj.weight", q0, q1, fdt),
                o_b=reader.get(b + "attn.c_proj.bias") if rank == 0 else None,
                up_w=reader.rows(b + "mlp.c_fc.weight", f0, f1, fdt), up_b=reader.get(b + "mlp.c_fc.bias")[f0:f1],
                down_w=reader.cols(b + "mlp.c_proj.weight", f0, f1, fdt),
                down_b=reader.get(b + "mlp.c_proj.bias") if rank == 0 else None,
            ))
        wte = reader.get("transformer.wte.weight")
        wpe = reader.get("transformer.wpe.weight")
        lnf_w, lnf_b = reader.get("transformer.ln_f.weight"), reader.get("transformer.ln_f.bias")
        head_w = reader.get("lm_head.weight") if (not cfg.tie_word_embeddings and reader.has("lm_head.weight")) else wte
        head_b = None
    elif mt == "llama":
        for i in range(cfg.num_layers):
            b = f"model.layers.{i}."
            a = b + "self_attn."
            d = dict(
                ln1_w=reader.get(b + "input_layernorm.weight"), ln2_w=reader.get(b + "post_attention_layernorm.weight"),
                qkv_w=torch.cat([reader.rows(a + "q_proj.weight", q0, q1, fdt), reader.rows(a + "k_proj.weight", k0, k1, fdt),
                                 reader.rows(a + "v_proj.weight", k0, k1, fdt)], 0),
                o_w=reader.cols(a + "o_proj.weight", q0, q1, fdt),
                gate_w=reader.rows(b + "mlp.gate_proj.weight", f0, f1, fdt),
                up_w=reader.rows(b + "mlp.up_proj.weight", f0, f1, fdt),
                down_w=reader.cols(b + "mlp.down_proj.weight", f0, f1, fdt),
            )
            if cfg.qkv_bias:
                d["qkv_b"] = torch.cat([reader.get(a + "q_proj.bias")[q0:q1], reader.get(a + "k_proj.bias")[k0:k1],
                                        reader.get(a + "v_proj.bias")[k0:k1]])
            if cfg.out_bias and rank == 0:
                d["o_b"] = reader.get(a + "o_proj.bias")
            layers.append(d)
        wte = reader.get("model.embed_tokens.weight")
        wpe = None
        lnf_w, lnf_b = reader.get("model.norm.weight"), None
        head_w = wte if cfg.tie_word_embeddings or not reader.has("lm_head.weight") else reader.get("lm_head.weight")
        head_b = None
    else:
        raise ValueError(mt)
    return _finish(cfg, plan, wte, wpe, layers, lnf_w, lnf_b, head_w, head_b, device, dtype, fp8)


# ------------------------------------------------------------------------------ per-rank shard cache
# a restart of a large TP deployment should not re-read, re-shard, re-interleave and
# re-quantize the HF checkpoint on every rank. The finished per-rank weights (this rank's shards,
# padded head, SwiGLU interleave, fp8 + scales) are written once as one safetensors file per rank
# and mmap-loaded by the native reader afterwards.
def _flat(mw: ModelWeights) -> Dict[str, torch.Tensor]:
    out: Dict[str, torch.Tensor] = {"wte": mw.wte, "lnf_w": mw.lnf_w}
    if mw.wpe is not None:
        out["wpe"] = mw.wpe
    if mw.lnf_b is not None:
        out["lnf_b"] = mw.lnf_b

    def put_lin(pfx, lin: Linear):
        out[pfx + ".w"] = lin.dense().contiguous()  # shards are stored row-major
        if lin.b is not None:
            out[pfx + ".b"] = lin.b
        if lin.w_scale is not None:
            out[pfx + ".s"] = lin.w_scale

    for i, L in enumerate(mw.layers):
        for nm in ("ln1_w", "ln1_b", "ln2_w", "ln2_b"):
            t = getattr(L, nm)
            if t is not None:
                out[f"l{i}.{nm}"] = t
        for nm in ("qkv", "o", "up", "down"):
            put_lin(f"l{i}.{nm}", getattr(L, nm))
    put_lin("head", mw.head)
    return out


def save_shard(mw: ModelWeights, path: str) -> None:
    from safetensors.torch import save_file

    # clone: a tied head is a view of the embedding table (safetensors refuses shared storage)
    tensors = {k: v.detach().cpu().contiguous().clone() for k, v in _flat(mw).items()}
    meta = {"format": "llmss_amd-shard-v1", "layers": str(len(mw.layers)),
            "glu": str(int(mw.layers[0].up.glu)) if mw.layers else "0",
            "rope_interleaved": str(int(mw.rope_interleaved))}
    if mw.head.w.untyped_storage().data_ptr() == mw.wte.untyped_storage().data_ptr():
        es = mw.wte.element_size()
        meta["tied_head_row"] = str((mw.head.w.data_ptr() - mw.wte.data_ptr()) // (es * mw.wte.shape[1]))
        meta["tied_table_rows"] = str(mw.wte.untyped_storage().nbytes() // (es * mw.wte.shape[1]))
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + f".tmp{os.getpid()}"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)  # atomic: a concurrent reader never sees a partial file


def load_shard(cfg: ModelConfig, path: str, device, dtype) -> ModelWeights:
    from ..utils.checkpoint import CheckpointReader

    rd = CheckpointReader([path])
    names = set(rd.routing)

    def get(name):
        if name not in names:
            return None
        t = rd.get(name)
        return t.to(device=device, dtype=dtype if t.is_floating_point() and t.dtype != torch.float32 else t.dtype)

    def lin(pfx, glu=False):
        s = rd.get(pfx + ".s").to(device) if pfx + ".s" in names else None
        w = rd.get(pfx + ".w").to(device)
        if s is None and w.is_floating_point():
            w = w.to(dtype)
        return Linear(w, get(pfx + ".b"), s, glu)

    layers = []
    for i in range(cfg.num_layers):
        layers.append(LayerWeights(get(f"l{i}.ln1_w"), get(f"l{i}.ln1_b"), get(f"l{i}.ln2_w"), get(f"l{i}.ln2_b"),
                                   lin(f"l{i}.qkv"), lin(f"l{i}.o"), lin(f"l{i}.up", glu=cfg.gated_mlp),
                                   lin(f"l{i}.down")))
    head, wte = lin("head"), get("wte")
    meta = rd.metadata()
    if "tied_head_row" in meta:  # re-tie: one [Vpadded, H] table, embedding and head shard are views of it
        lo, rows = int(meta["tied_head_row"]), int(meta["tied_table_rows"])
        table = torch.zeros(rows, wte.shape[1], dtype=wte.dtype, device=wte.device)
        table[:wte.shape[0]] = wte
        wte, head = table[:wte.shape[0]], Linear(table[lo:lo + head.w.shape[0]], head.b, head.w_scale, head.glu)
    mw = ModelWeights(wte=wte, wpe=get("wpe"), layers=layers, lnf_w=get("lnf_w"), lnf_b=get("lnf_b"), head=head,
                      rope_interleaved=meta.get("rope_interleaved", "0") == "1")
    if cfg.position == "rope":
        mw.cos, mw.sin = ref.rope_tables(cfg.max_position_embeddings, cfg.rotary_dim, cfg.rope_theta, device)
    return mw


def shard_cache_path(root: str, model_dir: str, files: List[str], tp: int, rank: int, dtype: torch.dtype,
                     fp8: bool) -> str:
    """Cache file for (checkpoint identity, TP layout, dtype); identity = paths + sizes + mtimes."""
    import hashlib

    h = hashlib.sha1(os.path.abspath(model_dir).encode())
    for f in sorted(files):
        st = os.stat(f)
        h.update(f"{os.path.basename(f)}:{st.st_size}:{int(st.st_mtime)}".encode())
    tag = str(dtype).replace("torch.", "") + ("-fp8" if fp8 else "")
    return os.path.join(root, h.hexdigest()[:16], f"tp{tp}-r{rank}-{tag}.safetensors")
