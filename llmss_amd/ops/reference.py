"""Plain-PyTorch definitions of every op (CPU execution path and the numerics oracle).

Each function has exactly the semantics of its gfx950 HIP kernel in ``llmss_amd/csrc`` and is
used (a) when the tensors live on the CPU (the TP=1 CPU plumbing configuration, gloo
multi-process tests) and (b) by the GPU tests as the fp32 reference. There is no runtime switch
from a GPU tensor to these functions: ``llmss_amd.ops`` routes by device only.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

ACTS = {"none": 0, "gelu_tanh": 1, "gelu": 2, "relu": 3, "silu_glu": 4}


def _act(x: torch.Tensor, act: str) -> torch.Tensor:
    if act in (None, "none"):
        return x
    if act == "gelu_tanh":
        return F.gelu(x, approximate="tanh")
    if act == "gelu":
        return F.gelu(x)
    if act == "relu":
        return F.relu(x)
    raise ValueError(act)


def add_norm(x, weight, bias, eps: float, rms: bool, residual: Optional[torch.Tensor] = None,
             ) -> Tuple[torch.Tensor, torch.Tensor]:
    """r = x (+ residual) [rounded to x.dtype]; y = norm(r) * w (+ b). Returns (y, r)."""
    r = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    rf = r.float()
    if rms:
        y = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps)
    else:
        mu = rf.mean(-1, keepdim=True)
        var = (rf - mu).pow(2).mean(-1, keepdim=True)
        y = (rf - mu) * torch.rsqrt(var + eps)
    y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype), r


def embed(ids: torch.Tensor, wte: torch.Tensor, positions: Optional[torch.Tensor] = None,
          wpe: Optional[torch.Tensor] = None) -> torch.Tensor:
    ids = ids.clamp(0, wte.shape[0] - 1)
    out = wte[ids]
    if wpe is not None:
        out = (out.float() + wpe[positions].float()).to(wte.dtype)
    return out


def rope_tables(max_pos: int, rot: int, theta: float, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, rot, 2, dtype=torch.float64) / rot))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return ang.cos().float().to(device), ang.sin().float().to(device)


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, rot: int,
               style: str) -> torch.Tensor:
    """x [T, H, D] -> rotated copy (first ``rot`` dims), fp32 math, x.dtype out."""
    xf = x.float()
    c = cos[positions][:, None, :]  # [T,1,rot/2]
    s = sin[positions][:, None, :]
    out = xf.clone()
    if style == "gptj":
        x0 = xf[..., 0:rot:2]
        x1 = xf[..., 1:rot:2]
        out[..., 0:rot:2] = x0 * c - x1 * s
        out[..., 1:rot:2] = x1 * c + x0 * s
    else:
        h = rot // 2
        x0 = xf[..., :h]
        x1 = xf[..., h:rot]
        out[..., :h] = x0 * c - x1 * s
        out[..., h:rot] = x1 * c + x0 * s
    return out.to(x.dtype)


def rope_cache(qkv: torch.Tensor, positions, cos, sin, k_cache, v_cache, slots, nh: int, nkv: int, D: int,
               rot: int, style: str, do_rope: bool = True) -> None:
    """In place: rotate q and k inside qkv; write rotated k and v to the paged cache at slots."""
    T = qkv.shape[0]
    q = qkv[:, : nh * D].view(T, nh, D)
    k = qkv[:, nh * D: (nh + nkv) * D].view(T, nkv, D)
    v = qkv[:, (nh + nkv) * D: (nh + 2 * nkv) * D].view(T, nkv, D)
    if do_rope and rot > 0:
        q.copy_(apply_rope(q, positions, cos, sin, rot, style))
        k.copy_(apply_rope(k, positions, cos, sin, rot, style))
    if k_cache is not None and slots is not None:
        bs = k_cache.shape[2]
        valid = slots >= 0
        sl = slots[valid]
        blk, off = sl // bs, sl % bs
        # cache [num_blocks, nkv, bs, D]
        k_cache[blk, :, off, :] = k[valid].to(k_cache.dtype)
        v_cache[blk, :, off, :] = v[valid].to(v_cache.dtype)


def attn_prefill(qkv: torch.Tensor, cu_seqlens, nh: int, nkv: int, D: int, scale: float) -> torch.Tensor:
    """Causal attention per packed sequence; q/k/v read from the fused qkv rows."""
    T = qkv.shape[0]
    out = torch.empty(T, nh * D, dtype=qkv.dtype, device=qkv.device)
    cu = [int(c) for c in (cu_seqlens.tolist() if torch.is_tensor(cu_seqlens) else cu_seqlens)]
    g = nh // nkv
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b == a:
            continue
        q = qkv[a:b, : nh * D].view(b - a, nh, D).float().transpose(0, 1)
        k = qkv[a:b, nh * D: (nh + nkv) * D].view(b - a, nkv, D).float().transpose(0, 1)
        v = qkv[a:b, (nh + nkv) * D: (nh + 2 * nkv) * D].view(b - a, nkv, D).float().transpose(0, 1)
        k = k.repeat_interleave(g, 0)
        v = v.repeat_interleave(g, 0)
        s = torch.matmul(q, k.transpose(1, 2)) * scale
        mask = torch.ones(b - a, b - a, dtype=torch.bool, device=qkv.device).tril()
        s = s.masked_fill(~mask, float("-inf"))
        p = torch.softmax(s, -1)
        o = torch.matmul(p, v).transpose(0, 1).reshape(b - a, nh * D)
        out[a:b] = o.to(qkv.dtype)
    return out


def gather_kv(cache: torch.Tensor, block_table_row: torch.Tensor, ctx: int) -> torch.Tensor:
    """Paged cache [nb, nkv, bs, D] -> contiguous [nkv, ctx, D] for one sequence."""
    bs = cache.shape[2]
    nblk = (ctx + bs - 1) // bs
    blocks = cache[block_table_row[:nblk].long()]  # [nblk, nkv, bs, D]
    return blocks.permute(1, 0, 2, 3).reshape(cache.shape[1], nblk * bs, cache.shape[3])[:, :ctx]


def attn_decode(q: torch.Tensor, k_cache, v_cache, block_tables, ctx_lens, nh: int, nkv: int, D: int,
                scale: float) -> torch.Tensor:
    """q [B, >= nh*D] (row-strided view allowed); returns [B, nh*D]."""
    B = q.shape[0]
    g = nh // nkv
    out = torch.empty(B, nh * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        ctx = int(ctx_lens[b])
        qq = q[b, : nh * D].view(nh, D).float()
        if ctx == 0:
            out[b] = 0
            continue
        k = gather_kv(k_cache, block_tables[b], ctx).float().repeat_interleave(g, 0)  # [nh, ctx, D]
        v = gather_kv(v_cache, block_tables[b], ctx).float().repeat_interleave(g, 0)
        s = torch.einsum("hd,htd->ht", qq, k) * scale
        p = torch.softmax(s, -1)
        out[b] = torch.einsum("ht,htd->hd", p, v).reshape(-1).to(q.dtype)
    return out


def attn_extend(q: torch.Tensor, k_cache, v_cache, block_tables, cu_q, ctx_lens, nh: int, nkv: int, D: int,
                scale: float) -> torch.Tensor:
    """Chunked prefill over the paged cache: sequence b's rows cu_q[b]:cu_q[b+1] sit at positions
    ctx_lens[b] - qlen ... ctx_lens[b] - 1 and attend every cached key up to their own position."""
    T = q.shape[0]
    g = nh // nkv
    out = torch.zeros(T, nh * D, dtype=q.dtype, device=q.device)
    cu = [int(c) for c in cu_q.tolist()]
    for b in range(len(cu) - 1):
        a, e = cu[b], cu[b + 1]
        if e == a:
            continue
        ctx = int(ctx_lens[b])
        p0 = ctx - (e - a)
        qq = q[a:e, : nh * D].view(e - a, nh, D).float().transpose(0, 1)  # [nh, q, D]
        k = gather_kv(k_cache, block_tables[b], ctx).float().repeat_interleave(g, 0)  # [nh, ctx, D]
        v = gather_kv(v_cache, block_tables[b], ctx).float().repeat_interleave(g, 0)
        s = torch.matmul(qq, k.transpose(1, 2)) * scale
        qpos = torch.arange(p0, ctx, device=q.device)[:, None]
        s = s.masked_fill(torch.arange(ctx, device=q.device)[None, :] > qpos, float("-inf"))
        out[a:e] = torch.matmul(torch.softmax(s, -1), v).transpose(0, 1).reshape(e - a, nh * D).to(q.dtype)
    return out


def glu_split(w_or_y: torch.Tensor, dim: int = -1):
    """Split a 16-row/column interleaved gate|up tensor into (gate, up)."""
    n = w_or_y.shape[dim]
    shp = list(w_or_y.shape)
    d = dim % len(shp)
    v = w_or_y.reshape(shp[:d] + [n // 32, 2, 16] + shp[d + 1:])
    gate = v.select(d + 1, 0).reshape(shp[:d] + [n // 2] + shp[d + 1:])
    up = v.select(d + 1, 1).reshape(shp[:d] + [n // 2] + shp[d + 1:])
    return gate, up


def glu_interleave(gate: torch.Tensor, up: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Inverse of :func:`glu_split`: [F, ...] x2 -> [2F, ...] interleaved in 16-row groups."""
    d = dim % gate.dim()
    F_ = gate.shape[d]
    if F_ % 16:
        raise ValueError("gated MLP width must be a multiple of 16 per rank")
    shp = list(gate.shape)
    g = gate.reshape(shp[:d] + [F_ // 16, 1, 16] + shp[d + 1:])
    u = up.reshape(shp[:d] + [F_ // 16, 1, 16] + shp[d + 1:])
    return torch.cat([g, u], dim=d + 1).reshape(shp[:d] + [2 * F_] + shp[d + 1:])


def dequant_fp8(w_q: torch.Tensor, w_scale: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    return (w_q.view(torch.float8_e4m3fn).float() * w_scale.float()[:, None]).to(dtype)


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, act: str = "none", glu: bool = False,
           w_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    wf = dequant_fp8(w, w_scale) if w_scale is not None else w.float()
    y = x.float() @ wf.t()
    if bias is not None:
        y = y + bias.float()
    if glu:
        g, u = glu_split(y, -1)
        y = F.silu(g) * u
    else:
        y = _act(y, act)
    return y.to(x.dtype)


def quant_fp8_rows(w: torch.Tensor):
    wf = w.float()
    amax = wf.abs().amax(dim=1).clamp_min(0)
    scale = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (wf / scale[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, scale


def sample(logits: torch.Tensor, temperature, top_k, top_p, seeds, generator=None) -> torch.Tensor:
    """Reference sampler: temperature -> top-k -> top-p -> multinomial (argmax if temp <= 0)."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.long, device=logits.device)
    for b in range(B):
        row = logits[b].float()
        t = float(temperature[b]) if temperature is not None else 0.0
        k = int(top_k[b]) if top_k is not None else 0
        p = float(top_p[b]) if top_p is not None else 1.0
        if not t > 0 or k == 1:
            out[b] = int(torch.argmax(row))
            continue
        x = row / t
        if 0 < k < V:
            kth = torch.topk(x, k).values[-1]
            x = x.masked_fill(x < kth, float("-inf"))
        if p < 1.0:
            probs = torch.softmax(x, -1)
            sp, si = probs.sort(descending=True)
            cum = sp.cumsum(0)
            keep = cum - sp < p  # keep tokens until mass >= p
            keep[0] = True
            thr = sp[keep].min()
            x = x.masked_fill(probs < thr, float("-inf"))
        probs = torch.softmax(x, -1)
        g = None
        if generator is not None:
            g = generator
        elif seeds is not None:
            g = torch.Generator(device="cpu")
            g.manual_seed(int(seeds[b]) & ((1 << 63) - 1))
        out[b] = int(torch.multinomial(probs.cpu(), 1, generator=g))
    return out


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Shifted LM loss as in the reference (gptj_modeling.py:612-622)."""
    return F.cross_entropy(logits[..., :-1, :].reshape(-1, logits.shape[-1]).float(),
                           labels[..., 1:].reshape(-1), ignore_index=-100)


def softmax_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
