"""Plain-PyTorch definitions of every op (CPU execution path and the numerics oracle).

Each function has exactly the semantics of its gfx950 HIP kernel in ``llmss_amd/csrc`` and is
used (a) when the tensors live on the CPU (the TP=1 CPU plumbing configuration, gloo
multi-process tests) and (b) by the GPU tests as the fp32 reference. There is no runtime switch
from a GPU tensor to these functions: ``llmss_amd.ops`` routes by device only.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
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


def rope_interleave_perm(D: int, rot: int) -> torch.Tensor:
    """Head-dim order that turns neox RoPE (pairs (j, j + rot/2)) into adjacent pairs (2j, 2j + 1): new
    dim 2j <- old j, 2j + 1 <- old j + rot/2, dims >= rot unchanged. Applied to the q and k rows of the
    fused QKV weight at load, attention scores are unchanged (q and k permute alike, V does not) and the
    rotation becomes the gptj form, which the QKV GEMM epilogue applies in-register for any tile width."""
    h = rot // 2
    first = torch.stack([torch.arange(h), torch.arange(h) + h], 1).reshape(-1)
    return torch.cat([first, torch.arange(rot, D)])


def rope_interleave_rows(t: torch.Tensor, nh: int, nkv: int, D: int, rot: int) -> torch.Tensor:
    """Permute the q and k head rows of a fused [(nh + 2 nkv) * D, ...] QKV weight / bias (see
    rope_interleave_perm); v rows stay."""
    perm = rope_interleave_perm(D, rot).to(t.device)
    nqk = (nh + nkv) * D
    idx = (torch.arange(nh + nkv, device=t.device)[:, None] * D + perm[None, :]).reshape(-1)
    out = t.clone()
    out[:nqk] = t[idx]
    return out


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


# fp8 KV cache rows: one (token, kv head) row = D e4m3 bytes + a 16-byte tail holding the row's fp32
# scale (bytes D..D+3; D+4..D+15 zero): scale = absmax / 448, value = e4m3 * scale. 16-B aligned rows,
# 0.56x the bytes of a bf16 row at D = 128.
KV8_TAIL = 16


def kv_rows_quant(x: torch.Tensor) -> torch.Tensor:
    """[..., D] float -> [..., D + 16] uint8 fp8 cache rows (csrc kernels: same arithmetic)."""
    xf = x.float()
    D = xf.shape[-1]
    amax = xf.abs().amax(-1, keepdim=True)
    sc = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (xf * (1.0 / sc)).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    rows = torch.zeros(*xf.shape[:-1], D + KV8_TAIL, dtype=torch.uint8, device=x.device)
    rows[..., :D] = q
    rows[..., D:D + 4] = sc.contiguous().view(torch.uint8)
    return rows


def kv_rows_dequant(rows: torch.Tensor, D: int) -> torch.Tensor:
    """[..., D + 16] uint8 fp8 cache rows -> [..., D] fp32."""
    q = rows[..., :D].contiguous().view(torch.float8_e4m3fn).float()
    sc = rows[..., D:D + 4].contiguous().view(torch.float32)
    return q * sc


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
        # cache [num_blocks, nkv, bs, D] (or fp8 rows [.., D + 16] uint8)
        if k_cache.dtype == torch.uint8:
            k_cache[blk, :, off, :] = kv_rows_quant(k[valid])
            v_cache[blk, :, off, :] = kv_rows_quant(v[valid])
        else:
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
    """Paged cache [nb, nkv, bs, D] -> contiguous [nkv, ctx, D] for one sequence (fp8 rows dequantised
    to fp32)."""
    bs = cache.shape[2]
    nblk = (ctx + bs - 1) // bs
    blocks = cache[block_table_row[:nblk].long()]  # [nblk, nkv, bs, D]
    out = blocks.permute(1, 0, 2, 3).reshape(cache.shape[1], nblk * bs, cache.shape[3])[:, :ctx]
    return kv_rows_dequant(out, cache.shape[3] - KV8_TAIL) if cache.dtype == torch.uint8 else out


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


def fake_quant_fp8_act(x: torch.Tensor) -> torch.Tensor:
    """Per-token e4m3 fake quantisation of GEMM activations, as the W8A8 path quantises them (csrc/quant.hip
    quant_fp8_rows_ld, the add_norm / attention fp8 twins): scale = absmax(row) / 448 (1 for a zero row),
    q = e4m3(clamp(x * (1 / scale), +-448)); returns q * scale in fp32."""
    xf = x.float()
    amax = xf.abs().amax(dim=-1, keepdim=True)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (xf * (1.0 / s)).clamp(-448, 448).to(torch.float8_e4m3fn).float()
    return q * s


def quant_mx_fp8(x: torch.Tensor):
    """OCP MX-fp8 of rows, as a W8A8 SwiGLU epilogue writes it for the down projection (csrc/common.h
    img_store_rows, mx_block_exp): per row and 32 columns the e8m0 scale 2^e with the smallest e such that the block's
    |max| / 2^e <= 448 (e clamped to [-126, 126]; 0 for an all-zero block), q = e4m3(x / 2^e). Returns (q uint8
    [M, K], s uint8 [M, K / 32] = e + 127)."""
    M, K = x.shape
    xb = x.float().reshape(M, K // 32, 32)
    amax = xb.abs().amax(-1)
    bits = (amax / 448.0).view(torch.int32)
    e = ((bits >> 23) & 255) - 127 + ((bits & 0x7FFFFF) != 0).to(torch.int32)
    e = torch.where(amax > 0, e.clamp(-126, 126), torch.zeros_like(e))
    q = (xb * torch.ldexp(torch.ones_like(amax), -e)[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).reshape(M, K), (e + 127).to(torch.uint8)


def dequant_mx_fp8(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    M, K = q.shape
    qf = q.view(torch.float8_e4m3fn).float().reshape(M, K // 32, 32)
    return (qf * torch.ldexp(torch.ones(s.shape), s.to(torch.int32) - 127)[..., None]).reshape(M, K)


def fake_quant_mx_act(x: torch.Tensor) -> torch.Tensor:
    """MX-fp8 fake quantisation (quant_mx_fp8 then back to fp32)."""
    return dequant_mx_fp8(*quant_mx_fp8(x))


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, act: str = "none", glu: bool = False,
           w_scale: Optional[torch.Tensor] = None, a8=False) -> torch.Tensor:
    """``a8`` (fp8 weights only): per-token e4m3 activations as well - the fp32 fake-quant oracle of W8A8;
    ``a8="mx"``: MX-fp8 activations (per-32 e8m0 block scales)."""
    wf = dequant_fp8(w, w_scale) if w_scale is not None else w.float()
    if a8 and w_scale is not None:
        xf = fake_quant_mx_act(x) if a8 == "mx" else fake_quant_fp8_act(x)
    else:
        xf = x.float()
    y = xf @ wf.t()
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


# ---------------------------------------------------------------------------------------- sampling
# CPU definition of the GPU sampler (csrc/sampling.hip sample_v3 / sample_cand): temperature ->
# top-k -> top-p -> Gumbel-max with Philox-4x32-10 noise keyed by (row seed, global token index).
# Top-p mass is summed as 2^-32 fixed-point integers, so the kept set does not depend on summation
# order - which is what lets a vocab-parallel (candidate) evaluation reproduce the full-row result.
def philox(idx: np.ndarray, seed: int) -> np.ndarray:
    """Philox-4x32-10 first output word for counters (idx, 0, 0, 0) and key = 64-bit seed."""
    m = np.uint64(0xFFFFFFFF)
    c0 = idx.astype(np.uint64) & m
    c1 = np.zeros_like(c0)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        h0, l0, h1, l1 = p0 >> np.uint64(32), p0 & m, p1 >> np.uint64(32), p1 & m
        c0, c1, c2, c3 = (h1 ^ c1 ^ k0) & m, l1, (h0 ^ c3 ^ k1) & m, l0
        k0, k1 = (k0 + np.uint64(0x9E3779B9)) & m, (k1 + np.uint64(0xBB67AE85)) & m
    return c0


def _mass(x: np.ndarray, mx: np.float32) -> np.ndarray:
    return (np.exp((x - mx).astype(np.float32)).astype(np.float32) * np.float32(4294967296.0)).astype(np.uint64)


def _select(x: np.ndarray, idx: np.ndarray, t: float, k: int, p: float, seed: int, V: int) -> int:
    """One row: x = scaled logits of the (candidate) elements, idx their global token ids."""
    valid = np.isfinite(x) | (x > -np.inf)
    x, idx = x[valid], idx[valid]
    if x.size == 0:
        return 0
    greedy = not t > 0 or k == 1
    thr = -np.inf
    if not greedy:
        order = np.lexsort((idx, -x))  # value desc, index asc
        xs = x[order]
        mx = np.float32(xs[0])
        if 0 < k < V and k <= xs.size:
            thr = xs[k - 1]
        if p < 1.0:
            kept = xs[xs >= thr]
            m = _mass(kept, mx)
            z = int(m.sum(dtype=np.uint64))
            target = max(1, int(float(p) * float(z)))
            cum = np.cumsum(m, dtype=np.uint64)
            j = int(np.searchsorted(cum, np.uint64(target), side="left"))
            tp = kept[min(j, kept.size - 1)]
            thr = max(thr, tp)
    v = x.astype(np.float32)
    if not greedy:
        keep = x >= thr
        v, idx = v[keep], idx[keep]
        r = philox(idx, seed)
        u = ((r >> np.uint64(8)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)
        v = (v - np.log(-np.log(u))).astype(np.float32)
    best = v.max()
    return int(idx[v == best].min())


def sample(logits: torch.Tensor, temperature, top_k, top_p, seeds, generator=None) -> torch.Tensor:
    """Full-row sampler (the GPU ``sample_v3`` definition): temperature -> top-k -> top-p -> Gumbel-max."""
    B, V = logits.shape
    lg = logits.detach().float().cpu().numpy()
    out = torch.empty(B, dtype=torch.long)
    for b in range(B):
        t = float(temperature[b]) if temperature is not None else 0.0
        k = int(top_k[b]) if top_k is not None else 0
        p = float(top_p[b]) if top_p is not None else 1.0
        sc = np.float32(1.0) if (not t > 0 or k == 1) else np.float32(1.0) / np.float32(t)
        x = lg[b].astype(np.float32) * sc
        seed = int(seeds[b]) & ((1 << 64) - 1) if seeds is not None else 0
        out[b] = _select(x, np.arange(V), t, k, p, seed, V)
    return out.to(logits.device)


def cand_topk(local: torch.Tensor, lo: int, V: int, temperature, top_k, K: int, KC: int) -> torch.Tensor:
    """Per-rank candidates of a vocab shard (GPU ``cand_topk``): every element whose scaled logit is
    >= the shard's K-th largest, packed per row as [KC values | KC global indices as int32 bits]."""
    B, vl = local.shape
    lg = local.detach().float().cpu().numpy()
    pack = np.zeros((B, 2 * KC), dtype=np.float32)
    for b in range(B):
        t = float(temperature[b]) if temperature is not None else 0.0
        k = int(top_k[b]) if top_k is not None else 0
        sc = np.float32(1.0) if (not t > 0 or k == 1) else np.float32(1.0) / np.float32(t)
        n = max(0, min(vl, V - lo))
        x = lg[b, :n].astype(np.float32) * sc
        kth = np.sort(x)[::-1][K - 1] if n >= K else -np.inf
        sel = np.flatnonzero(x >= kth)[:KC]
        vals = np.full(KC, -np.inf, dtype=np.float32)
        ids = np.full(KC, 0x7FFFFFFF, dtype=np.int32)
        vals[:sel.size] = x[sel]
        ids[:sel.size] = lo + sel
        pack[b, :KC] = vals
        pack[b, KC:] = ids.view(np.float32)
    return torch.from_numpy(pack).to(local.device)


def sample_cand(pack: torch.Tensor, groups: int, KC: int, temperature, top_k, top_p, seeds, V: int) -> torch.Tensor:
    """Sampling over gathered candidates [B, groups * 2KC] (GPU ``sample_cand``)."""
    B = pack.shape[0]
    a = pack.detach().cpu().numpy().reshape(B, groups, 2, KC)
    out = torch.empty(B, dtype=torch.long)
    for b in range(B):
        x = a[b, :, 0, :].reshape(-1).astype(np.float32)
        idx = a[b, :, 1, :].reshape(-1).view(np.int32).astype(np.int64)
        t = float(temperature[b]) if temperature is not None else 0.0
        k = int(top_k[b]) if top_k is not None else 0
        p = float(top_p[b]) if top_p is not None else 1.0
        seed = int(seeds[b]) & ((1 << 64) - 1) if seeds is not None else 0
        out[b] = _select(x, idx, t, k, p, seed, V)
    return out.to(pack.device)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Shifted LM loss as in the reference (gptj_modeling.py:612-622)."""
    return F.cross_entropy(logits[..., :-1, :].reshape(-1, logits.shape[-1]).float(),
                           labels[..., 1:].reshape(-1), ignore_index=-100)


def softmax_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
