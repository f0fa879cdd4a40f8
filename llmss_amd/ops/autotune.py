"""GEMM autotuner for the shapes an engine runs (decode batch buckets x layer projections).

The static planner in ``csrc/gemm.hip`` is a good default, but the best (kernel, tile, LDS ring
depth, split-K) choice for a memory-bound decode GEMM moves with M, N and K by 10-40% in ways a
rule does not capture (``bench/gemm_bench.py --sweep``). At engine start every decode shape is
timed over a candidate list and the winner goes into the native plan table, which every later
call (and HIP-graph capture) uses without hints.

Timing streams the weights from HBM the way a decode step does: candidates rotate over enough
weight copies (> 2x the 256 MiB Infinity Cache) that no call hits a cached tile. When the layer's
consumer reduces split-K partials itself (QKV -> rope, o/down -> add_norm at TP=1), the GEMM is
timed without its reduce and charged the consumer's extra slab reads instead.
"""
from __future__ import annotations

import itertools
import math
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..utils.logging import get_logger

log = get_logger(__name__)

_SLAB_READ_BPS = 4.0e12  # consumer-side fp32 partial reads (add_norm / rope), bytes/s
ILV_MIN_M = 128  # smallest M whose plans include the interleaved ring (profiles/r4_gemm/sweep512_ilv.log)
FINALISTS = 6  # candidates re-timed at full length after the short first round


@dataclass(frozen=True)
class GemmShape:
    N: int
    K: int
    glu: bool = False
    fp8: bool = False
    partial: bool = False  # consumer sums split-K slabs itself
    act: str = "none"


def candidates(M: int, N: int, K: int, glu: bool, fp8: bool) -> List[Tuple[int, int]]:
    """(nt_hint, split) pairs; nt_hint encodings are documented in csrc/gemm.hip launch_gemm."""
    out: List[Tuple[int, int]] = []
    splits = (1, 2, 4, 8)
    if fp8 or M <= 64:  # weight-streaming kernels (nt + 16 * variant); at M = 33-64 four 16-row MFMA tiles per wave
        out += [(nt + 16 * v, s) for v, nt, s in itertools.product((1, 2), (1, 2), splits)]
    if fp8:  # tiled kernel with fp8 weight tiles (no stream-K / big-tile variants)
        if M > 16:
            out += [((t | d) << 8, s) for t, d in ((3, 16), (3, 32), (2, 16), (2, 32)) for s in splits]
        if M >= 32:  # W8A8: per-token fp8 activations on the MX-fp8 matrix cores (ops/hip.py W8A8_FLAG)
            from .hip import W8A8_FLAG

            tiles = [3, 2] + ([1] if M > 64 else [])
            out += [(W8A8_FLAG | (t << 8) | (d << 12), s) for t in tiles for d in (2, 3, 4) for s in splits
                    if not (t == 1 and d > 3)]
            if K % 128 == 0:  # gemm_mid tiles with the fp8 MFMA (buffer-descriptor staging, csrc/gemm_mid.hip)
                mt = [11, 10, 13, 15, 7] + ([8, 12] if M > 64 else []) + ([9] if M >= 256 else [])
                out += [(W8A8_FLAG | (t << 8) | (d << 12), s) for t in mt for d in (3, 4)
                        for s in (1, 2, 3, 4, 5, 6, 8)]
                if M >= ILV_MIN_M:  # their software-pipelined k-loop (W8A8_ILV), 3-5 stages, 4-wave tiles
                    from .hip import W8A8_ILV

                    out += [(W8A8_FLAG | W8A8_ILV | (t << 8) | (d << 12), s) for t in mt if t not in (9, 12)
                            for d in (3, 4, 5) for s in (1, 2, 4) if (K // 128) // s >= 3]
            if M >= 256 and K % 128 == 0:
                out.append((W8A8_FLAG | (4 << 8), 1))
        return out
    # tiled: tile << 8 | depth code << 12   (tile 1: 128x128, 2: 64x128, 3: 64x64; depth 2/3/4/6)
    tiles = [(3, (0, 16, 32, 48)), (2, (0, 16, 32))]
    if M > 32:
        tiles.append((1, (0, 16)))
    for t, depths in tiles:
        for d in depths:
            out += [((t | d) << 8, s) for s in splits]
    if M > 32:  # stream-K (tile | depth | 128) << 8, split = workgroups per CU
        for t, d in ((1, 0), (1, 16), (2, 16), (2, 32), (3, 16), (3, 32)):
            out += [((t | d | 128) << 8, g) for g in (1, 2, 3)]
    if M >= 256 and K % 64 == 0:
        out.append((4 << 8, 1))
    if M >= 128:  # 8-wave 256x128 (5) / 256x64 (6) tiles: one workgroup per CU, deep split-K
        out += [((t | d) << 8, s) for t, d in ((5, 16), (6, 16), (6, 32)) for s in (2, 4, 8, 12, 16)]
    # gemm_mid (buffer-descriptor staging, csrc/gemm_mid.hip): 8 = 128x128, 9 = 256x128, 10 = 64x256,
    # 11 = 64x128, 12 = 128x256; depth code 16 / 32 = 3 / 4 stages (clamped to the LDS)
    mids = [(10, 16), (11, 16), (11, 32), (13, 16), (13, 32), (14, 32), (14, 48), (15, 16), (15, 32), (7, 32), (7, 48)]
    if M > 64:
        mids += [(8, 16), (8, 32), (12, 16)]
    if M >= 256:
        mids += [(9, 16)]
    # odd splits too: with one workgroup per CU the best grid lands just under a multiple of the 256 CUs
    # (64 x 256 tiles of a 12288-column QKV: 48 tiles x 5 = 240 workgroups)
    nk = -(-K // 64)
    out += [((t | d) << 8, s) for t, d in mids for s in (1, 2, 3, 4, 5, 6, 8, 11, 12) if s == 1 or nk // s >= 2]
    # K split over the waves of a workgroup, wave-private rings (hint bit 1024, csrc/gemm_dec.hip): M <= 64, column
    # widths 16-64, grids of 64-1024 workgroups (profiles/r6_dec: GPT-2-XL's up projection 9.9 vs 11.2 us)
    if M <= 64:
        for code, bn in ((1, 16), (2, 32), (3, 48), (4, 64)):
            tiles = -(-N // bn)
            out += [((code | 32 | 1024) << 8, s) for s in (1, 2, 3, 4, 5, 8, 10) if s <= nk and 64 <= tiles * s <= 1024]
            # (its in-launch split-K combine, hint bit 256, is selectable but not a candidate: 15.2 us at best for
            # GPT-2-XL's up projection against 10.6 unsplit, profiles/r6_dec)
    # interleaved ring (hint bit 512, csrc/gemm_mid.hip ILV): >= 3 stages
    if M >= ILV_MIN_M and K % 64 == 0:
        out += [((t | d | 512) << 8, s) for t, d in mids if d >= 16 for s in (1, 2, 3, 4, 5, 6, 8)
                if s == 1 or nk // s >= 3]
    # split-K combined inside the launch (hint bit 256, csrc/common.h splitk_combine): finished bf16
    # output with no reduce launch - for SwiGLU / activation GEMMs and row-parallel outputs that an
    # all-reduce needs whole; odd splits too (grid just under a multiple of the CU count)
    comb = [(3, 16), (2, 16), (11, 16), (10, 16), (13, 16), (14, 32), (15, 16), (7, 32)]
    if M > 64:
        comb += [(1, 0), (8, 16), (12, 16)]
    if M >= 256:
        comb += [(9, 0)]
    nk = -(-K // 64)
    out += [((t | d | 256) << 8, s) for t, d in comb for s in (2, 3, 4, 6, 8) if nk // s >= 2]
    return out


def _time(fn, iters: int) -> float:
    """GPU time per call. The calls are captured into one HIP graph and replayed (as the decode graphs
    run them): timing a host loop instead measures Python launch overhead (~10 us per call) for
    every kernel shorter than that, which is most TP-sharded decode GEMMs."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for i in range(iters):
            fn(i)
    g.replay()
    best = float("inf")
    for _ in range(2):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)  # us
    return best


def tune_shape(M: int, shape: GemmShape, device, weight_budget: int = 600 << 20, iters: int = 16,
               cands: Optional[Sequence[Tuple[int, int]]] = None,
               copies: Optional[int] = None) -> Tuple[int, int, float, float]:
    """Best (nt_hint, split, us, default_us) for one shape (``copies``: weight copies to rotate over instead
    of enough to exceed ``weight_budget``; 1 = cache-resident weights, a diagnostic)."""
    from . import hip as H

    N, K = shape.N, shape.K
    wbytes = N * K * (1 if shape.fp8 else 2)
    ncopy = copies or max(2, min(64, math.ceil(weight_budget / wbytes)))
    g = torch.Generator(device=device)
    g.manual_seed(1234)
    x = (torch.randn(M, K, device=device, generator=g) * 0.5).to(torch.bfloat16)
    if shape.fp8:
        base = torch.randint(0, 120, (N, K), device=device, dtype=torch.uint8, generator=g)
        ws = [base.clone() for _ in range(ncopy)]
        sc = torch.full((N,), 1e-2, device=device)
    else:
        base = (torch.randn(N, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
        ws = [base.clone() for _ in range(ncopy)]
        sc = None
    nout = N // 2 if shape.glu else N
    y = torch.empty(M, nout, dtype=torch.bfloat16, device=device)
    partial = shape.partial and not shape.glu and shape.act in ("none", None)

    def run(nt, s):
        def f(i):
            r = H.linear(x, ws[i % ncopy], None, shape.act, shape.glu, sc, out=None if partial else y,
                         nt_hint=nt, split_hint=s, partial_ok=partial)
            return r
        return f

    def cost(nt, s, n=iters):
        f = run(nt, s)
        r = f(0)
        slabs = r.S if isinstance(r, H.PartialSum) else 0
        for i in range(2):
            f(i)
        torch.cuda.synchronize(device)
        t = _time(f, n)
        return t + (slabs * M * N * 4 / _SLAB_READ_BPS * 1e6 if slabs else 0.0)

    default = cost(0, 0)
    best = (0, 0, default)
    if cands is None:
        cands = candidates(M, N, K, shape.glu, shape.fp8)
    # two rounds (engine start-up time): every candidate on a short graph (4 calls), then the
    # FINALISTS fastest of them again at the full `iters` - a short graph ranks plans that differ by > ~3 % the
    # same way, and the final choice is made on the long timings only
    quick = []
    for nt, s in cands:
        try:
            quick.append((cost(nt, s, 4), nt, s))
        except (ValueError, RuntimeError):  # config rejected by host-side validation
            continue
    quick.sort()
    for _, nt, s in quick[:FINALISTS]:
        t = cost(nt, s)
        if t < best[2] * 0.98:  # prefer the static plan unless a candidate is clearly faster
            best = (nt, s, t)
    del ws
    return best[0], best[1], best[2], default


def model_shapes(model) -> Dict[str, GemmShape]:
    """The per-layer projections of a DecoderLM (layer 0 is representative) + the LM head."""
    L = model.w.layers[0]
    fuse = model.tp.size == 1 and not model.cfg.parallel_block
    act = model.act if not L.up.glu else "none"
    def shp(lin, partial, act_="none"):
        return GemmShape(lin.N, lin.K, lin.glu, lin.w_scale is not None, partial, act_)

    out = {"qkv": shp(L.qkv, True), "o": shp(L.o, fuse), "up": shp(L.up, False, act), "down": shp(L.down, fuse)}
    out["head"] = shp(model.w.head, False)
    # the column-chunked decode schedule's slices of o / down (DecoderLM._reduce_cols): whenever it may run - forced,
    # or a candidate of the engine's capture-time A/B on a real communicator - so the A/B compares tuned plans
    col_mode = getattr(model, "col_mode", "0")
    if (not model.cfg.parallel_block and (col_mode == "force" or (col_mode == "auto" and model.tp.is_real))
            and model.col_ok(L.o) and model.col_ok(L.down)):
        C = model.col_chunks
        out["o_col"] = GemmShape(L.o.N // C, L.o.K, False, L.o.w_scale is not None, False, "none")
        out["down_col"] = GemmShape(L.down.N // C, L.down.K, False, L.down.w_scale is not None, False, "none")
    return out


def qkv_epi_candidates(M: int, N: int, K: int, D: int, neox_rope: bool) -> List[Tuple[int, int]]:
    """(nt_hint, split) plans that can run the QKV RoPE + KV-write epilogue: tiled / gemm_mid tiles, unsplit
    or combined in-launch (a split plan runs as a combine); neox RoPE needs head-aligned tiles (BN % D)."""
    tiles = [(3, 64, (16, 32)), (2, 128, (16, 32)), (11, 128, (16, 32)), (10, 256, (16,)), (13, 192, (16, 32)), (14, 32, (32, 48)), (15, 96, (16, 32)), (7, 48, (32, 48))]
    if M > 64:
        tiles += [(1, 128, (0, 16)), (8, 128, (16,)), (12, 256, (16,))]
    if M >= 256:
        tiles += [(9, 128, (0,))]
    nk = -(-K // 64)
    out = []
    if M <= 64:  # the K-split-wave decode kernel (csrc/gemm_dec.hip), unsplit (its in-launch combine measured slower)
        out += [((code | 32 | 1024) << 8, 1) for code, bn in ((1, 16), (2, 32), (3, 48), (4, 64))
                if not (neox_rope and bn % D)]
    for t, bn, depths in tiles:
        if neox_rope and bn % D:
            continue
        for d in depths:
            out += [((t | d | (256 if s > 1 else 0)) << 8, s) for s in (1, 2, 3, 4, 6, 8) if s == 1 or nk // s >= 2]
    return out


def tune_qkv_epilogue(model, ms: Sequence[int], native=None, iters: int = 16) -> Dict[int, Tuple[float, float]]:
    """Per decode bucket M: GEMM + rope_cache (the tuned QKV plan, its slabs summed by the rope kernel) vs
    the fused QKV GEMM whose epilogue applies RoPE and writes the paged KV cache (hip.linear_qkv). Where the
    fused launch is faster its plan goes into the native table as kind 3, which the decoder's QKV step
    consults. Returns {M: (unfused us, fused us)}."""
    from .. import _native
    from . import hip as H

    lib = native or _native()
    cfg, p, L = model.cfg, model.plan, model.w.layers[0]
    if L.qkv.w_scale is not None or getattr(model, "kv_fp8", False):
        return {}
    dev = model.device
    N, K, D = L.qkv.N, L.qkv.K, cfg.head_dim
    do_rope = cfg.position == "rope"
    rot, style = cfg.rotary_dim, cfg.rope_style
    neox = do_rope and style != "gptj"
    ncopy = max(2, min(64, math.ceil((600 << 20) / (N * K * 2))))
    g = torch.Generator(device=dev)
    g.manual_seed(4321)
    base = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    ws = [base.clone() for _ in range(ncopy)]
    bias = L.qkv.b
    res = {}
    for M in sorted(set(int(m) for m in ms)):
        bs = 16
        nb = -(-M // bs) + 1
        kc = torch.zeros(nb, p.nkv_l, bs, D, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        slots = torch.arange(M, device=dev, dtype=torch.int64)
        pos = torch.arange(M, device=dev, dtype=torch.int64) % min(cfg.max_position_embeddings, 256)
        x = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)

        def unfused(i):
            q = H.linear(x, ws[i % ncopy], bias, partial_ok=True)
            H.rope_cache(q, pos, model.w.cos, model.w.sin, kc, vc, slots, p.nh_l, p.nkv_l, D, rot, style, do_rope)

        def fused_fn(nt, s):
            def f(i):
                y = H.linear_qkv(x, ws[i % ncopy], bias, pos, model.w.cos, model.w.sin, kc, vc, slots, p.nh_l,
                                 p.nkv_l, D, rot, style, do_rope, nt_hint=nt, split_hint=s)
                if y is None:
                    raise RuntimeError("plan cannot take the QKV epilogue")
            return f

        unfused(0)
        torch.cuda.synchronize(dev)
        t_un = _time(unfused, iters)
        best = (0, 0, float("inf"))
        for nt, s in qkv_epi_candidates(M, N, K, D, neox):
            try:
                f = fused_fn(nt, s)
                f(0)
                torch.cuda.synchronize(dev)
                t = _time(f, iters)
            except (RuntimeError, ValueError):
                continue
            if t < best[2]:
                best = (nt, s, t)
        if best[0] and best[2] < t_un * 0.98:
            lib.gemm_tuned_set(M, N, K, False, 3, best[0], best[1])
            _QKV_PLANS[(M, N, K)] = (best[0], best[1])
        res[M] = (t_un, best[2])
    del ws
    log.info("QKV RoPE/KV-write epilogue: %s", ", ".join(
        f"M={m} {'fused' if f < u * 0.98 else 'unfused'} {min(u, f):.1f}us (unfused {u:.1f})" for m, (u, f) in res.items()))
    return res


# process-wide results: a second engine in the same process reuses the first one's plans, so both
# run bit-identical kernels (and skip the tuning time)
_DONE: Dict[Tuple[int, GemmShape, str], Tuple[int, int, float, float]] = {}
_QKV_DONE: Dict[tuple, Dict[int, Tuple[float, float]]] = {}
_QKV_PLANS: Dict[tuple, Tuple[int, int]] = {}


def _reinstall_qkv(lib, model, results):
    L = model.w.layers[0]
    for M in results:
        plan = _QKV_PLANS.get((M, L.qkv.N, L.qkv.K))
        if plan:
            lib.gemm_tuned_set(M, L.qkv.N, L.qkv.K, False, 3, plan[0], plan[1])


def representatives(ms: Sequence[int]) -> Dict[int, int]:
    """Row count whose tuned plan each decode size uses: every size up to 64 is tuned itself (the K-split-wave
    kernel's 16 / 32 / 64-row variants and the streaming kernels change plans there); above 64 every other size,
    counted down from the largest, and the sizes in between take the plan of the next larger tuned size (a plan is
    valid at any M; the 96-512-row buckets of a TP=8 engine differ by <= 25 % in M). Halves the tuning time of a
    TP=8 engine's large buckets."""
    ms = sorted(set(int(m) for m in ms))
    out = {m: m for m in ms if m <= 64}
    big = [m for m in ms if m > 64][::-1]
    for i, m in enumerate(big):
        out[m] = m if i % 2 == 0 else big[i - 1]
    return out


def tune_model(model, ms: Sequence[int], native=None) -> Dict[Tuple[str, int], Tuple[int, int, float, float]]:
    """Tune every (shape, M) pair and install the winners in the native plan table."""
    from .. import _native

    lib = native or _native()
    dev = model.device
    t0 = time.perf_counter()
    res = {}
    done = _DONE
    rep = representatives(ms)
    for name, shp in model_shapes(model).items():
        for M in sorted(set(int(m) for m in ms)):
            if name.endswith("_col") and getattr(model, "col_mode", "0") != "force" and M < model.col_min:
                continue  # column chunks run only in the buckets the capture-time A/B tries them on
            key = (rep[M], shp, str(dev))
            if key not in done:
                done[key] = tune_shape(rep[M], shp, dev)
            nt, s, t, t0_us = done[key]
            if nt:
                lib.gemm_tuned_set(M, shp.N, shp.K, shp.glu, int(shp.fp8), nt, s)
            res[(name, M)] = done[key]
    # the fused QKV epilogue is a candidate wherever it applies (tune_qkv_epilogue decides per bucket)
    key = ("qkv_epi", tuple(sorted(set(int(m) for m in ms))), model_shapes(model)["qkv"], str(dev),
           model.cfg.head_dim, model.cfg.rotary_dim, model.cfg.rope_style, model.cfg.position)
    if key not in _QKV_DONE:
        _QKV_DONE[key] = tune_qkv_epilogue(model, ms, lib)
    else:  # re-install this process's earlier winners
        _reinstall_qkv(lib, model, _QKV_DONE[key])
    for M, (u, f) in _QKV_DONE[key].items():
        res[("qkv_epi", M)] = (0, 0, min(u, f), u)
    torch.cuda.synchronize(dev)
    gain = sum(v[3] - v[2] for v in res.values())
    log.info("autotuned %d GEMM shapes in %.1fs (sum of per-call gains %.1f us)", len(res),
             time.perf_counter() - t0, gain)
    return res
