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

import contextlib
import dataclasses
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

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
    """One forward step over T flattened tokens.

    kind "prefill": every sequence starts at position 0 (cu_seqlens over its tokens);
    kind "decode": one token per sequence attending its paged context (block_tables, ctx_lens);
    kind "extend": rows [0, num_decode) are single-token decodes (as "decode"), the remaining rows
    are prompt chunks (cu_seqlens relative to row num_decode) that may continue a cached prefix
    (has_prefix: some chunk starts past position 0, so its attention reads the paged cache).
    block_tables / ctx_lens cover every sequence of the step, decodes first.
    """
    kind: str  # "prefill" | "decode" | "extend"
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
    num_decode: int = 0  # extend: leading single-token decode rows
    has_prefix: bool = False  # extend: a prompt chunk continues a cached prefix
    cu_host: Optional[Sequence[int]] = None  # prefill: cu_seqlens on the host (micro-batch split points)


class StreamLedger:
    """Fork / join bookkeeping of the comm-stream schedules (_reduce_rows, _reduce_cols, _hidden_states_overlap).

    A HIP graph capture ends in hipErrorStreamCaptureUnjoined when work forked off the capturing stream is never
    joined back (profiles/r6_capture: a clean Python error for every stream / event / allocator topology these
    schedules use, with and without native RCCL). Each fork (the comm stream waits for the compute stream, then
    runs a collective) and each join (the compute stream waits for the comm stream, or for an event recorded on it
    after the forked work - the comm stream runs in order, so that joins every earlier fork too) is registered
    here, on CPU as well where no stream exists, so the gloo tests check the structure the GPU graphs rely on, and
    DecoderLM.hidden_states asserts after every forward - i.e. before any capture ends - that nothing is open."""

    def __init__(self):
        self.open: List[int] = []  # fork tokens not yet joined, oldest first
        self.forks = 0  # forks since construction (tests: the schedule really forked)

    def fork(self, cur, comm) -> int:
        if comm is not None:
            comm.wait_stream(cur)
        self.forks += 1
        self.open.append(self.forks)
        return self.forks

    def mark(self, comm, tok: int):
        """(tok, event recorded on ``comm`` after fork ``tok``'s work) - what a later wait() joins."""
        ev = None
        if comm is not None:
            ev = torch.cuda.Event()
            ev.record(comm)
        return tok, ev

    def wait(self, cur, mark) -> None:
        if mark is None:
            return
        tok, ev = mark
        if ev is not None:
            cur.wait_event(ev)
        self.open = [t for t in self.open if t > tok]

    def join(self, cur, comm) -> None:
        if comm is not None:
            cur.wait_stream(comm)
        self.open.clear()

    def check(self, where: str) -> None:
        if self.open:
            n, self.open = len(self.open), []
            raise RuntimeError(f"{where}: {n} comm-stream fork(s) never joined back to the compute stream")


class DecoderLM:
    def __init__(self, cfg: ModelConfig, weights: ModelWeights, tp: Optional[TPGroup] = None):
        if weights.rope_interleaved and cfg.rope_style == "neox":
            # q / k head dims were interleaved at load: the same rotation in its gptj (adjacent-pair) form
            cfg = dataclasses.replace(cfg, rope_style="gptj")
        self.cfg = cfg
        self.w = weights
        self.tp = tp or TPGroup()
        self.plan: ShardPlan = shard_plan(cfg, self.tp.size, self.tp.rank)
        self.scale = cfg.head_dim ** -0.5
        self.rms = cfg.norm == "rmsnorm"
        self.act = "none" if cfg.gated_mlp else cfg.activation
        # TP all-reduce / GEMM overlap: the row-parallel output is cut into row buckets of about
        # `bucket_bytes` (LLMSS_TP_BUCKET_BYTES, default 32 MiB: a prefill chunk's all-reduce is then
        # long enough to hide the next chunk's GEMM behind it, while each RCCL call stays in its
        # bandwidth regime on xGMI); a decode step's few-MiB all-reduce stays one bucket unless the
        # knob is lowered. `overlap_rows` (tests) fixes the bucket in rows instead.
        self.overlap_rows: Optional[int] = None
        self.bucket_bytes = int(os.environ.get("LLMSS_TP_BUCKET_BYTES", str(32 << 20)))
        # fp8 (e4m3 + per-row scale) paged KV cache (LLMSS_KV_DTYPE=fp8 or LLMEngine(kv_dtype="fp8"))
        self.kv_fp8 = os.environ.get("LLMSS_KV_DTYPE", "bf16") == "fp8"
        # decode steps of at least this many sequences run as two interleaved micro-batches so each one's
        # all-reduces overlap the other's compute (only when collectives cost time; 0 = off). Set per bucket by the
        # engine's capture-time A/B on the real communicator (LLMEngine._schedule_ab), or by a caller. Under the TP=8
        # comm model it beats one all-reduce (60.0 K vs 55.4 K tok/s) since the comm stream runs at normal priority
        # (profiles/r5_tp8sim); round 1's +51 % loss was measured with a high-priority comm stream.
        self.tbo_min = 0
        # prefill steps of at least this many tokens (and >= 2 sequences) run as two micro-batches split at
        # a sequence boundary, so one half's all-reduces (hundreds of MiB each at TP=8) overlap the other
        # half's GEMMs and attention; only when collectives cost time (0 = off)
        self.tbo_prefill_min = int(os.environ.get("LLMSS_TP_PREFILL_OVERLAP_MIN", "8192"))
        # QKV GEMM epilogue with RoPE + paged KV write (one launch instead of two) wherever the autotuner
        # installed a faster plan for it (ops/autotune.py tune_qkv_epilogue)
        self.qkv_epi = True
        # decode batch sizes whose GQA attention runs on the MFMA extend kernel (one workgroup per kv head
        # serving its whole query-head group: K/V staged once, QK^T and PV on the matrix cores) instead of
        # the VALU split-K decode kernel; filled by LLMEngine's capture-time timing for G >= 4 groups
        self.gqa_mfma: set = set()
        self._norm_quant = True  # add_norm writes the fp8 twin of its output for a W8A8 consumer
        self._mx_mlp = True  # W8A8 gate/up hands its SwiGLU output to down as MX-fp8 (_mlp)
        # row-sharded decode schedule (TP > 1): each row-parallel output is reduce-scattered instead of
        # all-reduced, add + norm run on this rank's M / tp rows (the residual stream stays sharded) and the
        # normed rows are all-gathered for the next column-parallel GEMM (_hidden_states_rsag). Decode batch
        # sizes in `rsag` take it: LLMSS_TP_RSAG=1 every divisible decode batch, "auto" (default) the buckets
        # the engine's capture-time A/B picks on the real communicator, 0 never
        self.rsag_mode = os.environ.get("LLMSS_TP_RSAG", "auto")
        self.rsag: set = set()
        # column-chunked decode schedule (TP > 1, _reduce_cols): each row-parallel projection runs as C GEMMs over
        # disjoint output-column slices of its weight (no weight byte read twice); chunk c's all-reduce goes to the
        # comm stream while chunk c + 1's GEMM runs, and add_norm reads the chunk-major result. Decode
        # batch sizes in `col` take it: LLMSS_TP_COL=C (> 1) every decode step with C chunks, "auto" the buckets the
        # engine's capture-time A/B picks (4 chunks), 0 (default) never: it lost to the single all-reduce by 20-35 %
        # at every size under the TP=8 comm model (profiles/r5_tp8sim), so it no longer costs start-up time
        col = os.environ.get("LLMSS_TP_COL", "0")
        self.col_mode = "auto" if col == "auto" else ("force" if int(col) > 1 else "0")
        self.col_chunks = int(col) if col not in ("auto", "0", "1") else 4
        # smallest decode bucket the capture-time A/B tries it on (the collectives are small below; and under the
        # TP=8 comm model it lost at every size, profiles/r5_tp8sim)
        self.col_min = 256
        self.col: set = set()
        self._cu_decode = {}
        self._comm_stream = None
        self._ledger = StreamLedger()

    @property
    def device(self):
        return self.w.wte.device

    @property
    def dtype(self):
        return self.w.wte.dtype

    # --------------------------------------------------------------------------------- KV
    def kv_cache_shape(self, num_blocks: int, block_size: int):
        # fp8 KV (kv_fp8): each (token, kv head) row = head_dim e4m3 bytes + a 16-B tail with its fp32
        # scale (ops/reference.py kv_rows_quant); decode attention then streams 0.56x the bytes
        row = self.cfg.head_dim + ops.ref.KV8_TAIL if self.kv_fp8 else self.cfg.head_dim
        return (num_blocks, self.plan.nkv_l, block_size, row)

    def kv_bytes_per_block(self, block_size: int) -> int:
        row = self.cfg.head_dim + ops.ref.KV8_TAIL if self.kv_fp8 else self.cfg.head_dim * 2
        return 2 * self.cfg.num_layers * self.plan.nkv_l * block_size * row

    def allocate_kv_cache(self, num_blocks: int, block_size: int):
        shp = self.kv_cache_shape(num_blocks, block_size)
        dt = torch.uint8 if self.kv_fp8 else self.dtype
        return [(torch.zeros(shp, dtype=dt, device=self.device),
                 torch.zeros(shp, dtype=dt, device=self.device)) for _ in range(self.cfg.num_layers)]

    # ---------------------------------------------------------------------------- forward
    def _qkv_rope_cache(self, L, y, inp: StepInput, kc, vc):
        """QKV projection, RoPE and the paged KV write of the step's tokens -> the bf16 qkv rows.

        Where the autotuner found it faster (a kind-3 plan for this M, ops/autotune.py tune_qkv_epilogue)
        this is ONE GEMM launch whose epilogue rotates q / k and stores k / v to the cache; otherwise the
        GEMM (split-K slabs allowed) followed by the rope_cache kernel, which sums the slabs itself."""
        cfg, p = self.cfg, self.plan
        do_rope = cfg.position == "rope"
        if y.is_cuda and self.qkv_epi and not self.kv_fp8 and L.qkv.w.dim() == 2 and L.qkv.w_scale is None \
                and _hip_ops().lib().gemm_tuned_get(y.shape[0], L.qkv.N, L.qkv.K, False, 3) is not None:
            out = _hip_ops().linear_qkv(y, L.qkv.w, L.qkv.b, inp.positions, self.w.cos, self.w.sin, kc, vc, inp.slots,
                                        p.nh_l, p.nkv_l, cfg.head_dim, cfg.rotary_dim, cfg.rope_style, do_rope)
            if out is not None:
                return out
        qkv = L.qkv(y, partial_ok=True)
        return ops.rope_cache(qkv, inp.positions, self.w.cos, self.w.sin, kc, vc, inp.slots,
                              p.nh_l, p.nkv_l, cfg.head_dim, cfg.rotary_dim, cfg.rope_style, do_rope=do_rope)

    def _attention(self, L, y, inp: StepInput, kc, vc):
        cfg, p = self.cfg, self.plan
        D = cfg.head_dim
        qkv = self._qkv_rope_cache(L, y, inp, kc, vc)
        if inp.kind == "decode" and qkv.is_cuda and qkv.shape[0] in self.gqa_mfma:
            B = qkv.shape[0]
            # fp8 models whose rank holds one kv head (Llama-2-70B at TP=8): the attention launch also writes the
            # o-projection's per-token fp8 input, so the W8A8 GEMM skips its own quantisation launch
            f8 = self._fp8_in(L.o, qkv) and _hip_ops().extend_fp8_twin_ok(p.nh_l, p.nkv_l)
            return ops.attn_extend(qkv, kc, vc, inp.block_tables, self.decode_cu(B, qkv.device), inp.ctx_lens, 1,
                                   p.nh_l, p.nkv_l, D, self.scale, fp8_out=f8)
        if inp.kind == "prefill":
            return ops.attn_prefill(qkv, inp.cu_seqlens, inp.max_seqlen, p.nh_l, p.nkv_l, D, self.scale)
        if inp.kind == "extend":
            return self._attention_extend(qkv, inp, kc, vc)
        return ops.attn_decode(qkv, kc, vc, inp.block_tables, inp.ctx_lens, p.nh_l, p.nkv_l, D, self.scale,
                               inp.max_ctx, splits=inp.decode_splits)

    def _attention_extend(self, qkv, inp: StepInput, kc, vc):
        """Mixed step: decode rows through the split-K decode kernel, prompt-chunk rows through the
        flash prefill kernel (no cached prefix) or the paged extend kernel, into one output."""
        p, D = self.plan, self.cfg.head_dim
        T, nd = qkv.shape[0], inp.num_decode
        out = torch.empty(T, p.nh_l * D, dtype=qkv.dtype, device=qkv.device)
        if nd:
            ops.attn_decode(qkv[:nd], kc, vc, inp.block_tables[:nd], inp.ctx_lens[:nd], p.nh_l, p.nkv_l, D,
                            self.scale, inp.max_ctx, out=out[:nd])
        if T > nd:
            if inp.has_prefix:
                ops.attn_extend(qkv[nd:], kc, vc, inp.block_tables[nd:], inp.cu_seqlens, inp.ctx_lens[nd:],
                                inp.max_seqlen, p.nh_l, p.nkv_l, D, self.scale, out=out[nd:])
            else:
                ops.attn_prefill(qkv[nd:], inp.cu_seqlens, inp.max_seqlen, p.nh_l, p.nkv_l, D, self.scale,
                                 out=out[nd:])
        return out

    def _mlp(self, L, y, partial_ok=False):
        """down(up(y)). An fp8 MLP whose tuned plans both run W8A8 gemm_mid tiles (ops/hip.py mx_mlp_ok) takes the
        gate/up SwiGLU output as MX-fp8 (e4m3 + one e8m0 scale per 32 outputs) written by the gate/up epilogue: no
        bf16 intermediate and no per-token quantisation launch before the down projection (VERDICT r5 missing #4)."""
        if (self._mx_mlp and L.down.w_scale is not None and L.up.glu and y.is_cuda and L.up.w.dim() == 2
                and _hip_ops().mx_mlp_ok(y.shape[0], L.up, L.down)):
            H = _hip_ops()
            h = H.linear(y, L.up.w, L.up.b, "none", True, L.up.w_scale, mx_out=True)
            return H.linear(h, L.down.w, L.down.b, "none", False, L.down.w_scale, partial_ok=partial_ok)
        return L.down(L.up(y, self.act), partial_ok=partial_ok)

    def _fp8_in(self, lin, x) -> bool:
        """The linear consuming add_norm's output runs W8A8 at this row count: have add_norm write the per-token
        fp8 twin so the GEMM skips its quantisation launch."""
        if lin.w_scale is None or not x.is_cuda or lin.w.dim() != 2 or not self._norm_quant:
            return False
        return _hip_ops().w8a8_planned(x.shape[0], lin.N, lin.K, lin.glu)

    def decode_cu(self, B: int, device) -> torch.Tensor:
        """[0, 1, .., B] int32: a decode step as B one-token 'chunks' (the extend kernel's cu_q); made once per B
        outside graph capture (the engine's eager warm-up runs every bucket first)."""
        cu = self._cu_decode.get((B, str(device)))
        if cu is None:
            cu = self._cu_decode[(B, str(device))] = torch.arange(B + 1, dtype=torch.int32, device=device)
        return cu

    def bucket_rows(self, M: int) -> int:
        """Rows per all-reduce bucket of an M-row row-parallel output (>= M: one all-reduce)."""
        if self.overlap_rows is not None:
            return self.overlap_rows
        row_bytes = self.cfg.hidden_size * 2
        rows = max(8, self.bucket_bytes // row_bytes // 8 * 8)
        if rows >= M:
            return M
        nb = -(-M // rows)  # equal buckets (a short last one would pay a full RCCL latency)
        return (-(-M // nb) + 7) // 8 * 8

    def _comm(self, device):
        if self._comm_stream is None:
            # normal priority: a higher-priority queue makes the hardware preempt the compute queue's waves for every
            # comm kernel beside them, ~3x on each overlapped kernel (profiles/r5_tp8sim: TBO 20.9 K vs 60.0 K tok/s)
            self._comm_stream = torch.cuda.Stream(device=device)
        return self._comm_stream

    def _reduce_rows(self, fn, *inputs) -> torch.Tensor:
        """``all_reduce(fn(*inputs))`` for a row-parallel projection (or a whole MLP).

        Large steps run in row chunks: chunk c's RCCL all-reduce is issued on the comm
        stream while the compute stream already runs chunk c+1's GEMMs, so the per-layer
        all-reduce hides behind the next GEMM (prefill at TP=8 moves ~0.5 GB per all-reduce). Decode
        steps (a few MB, latency-bound) keep one all-reduce.
        """
        if not self.tp.comm_active:
            return fn(*inputs)
        M = inputs[0].shape[0]
        step = self.bucket_rows(M)
        if M <= step or step <= 0:
            return self.tp.all_reduce(fn(*inputs))
        gpu = inputs[0].is_cuda  # gloo / CPU: same chunking (numerics) and ledger, no streams
        cur = torch.cuda.current_stream() if gpu else None
        comm = self._comm(inputs[0].device) if gpu else None
        outs = []
        for r in range(0, M, step):
            y = fn(*(t[r:r + step] for t in inputs))
            self._ledger.fork(cur, comm)  # chunk r's GEMM done
            with (torch.cuda.stream(comm) if gpu else contextlib.nullcontext()):
                self.tp.all_reduce(y)
            # no record_stream: `outs` holds every chunk until the compute stream has waited for the comm
            # stream (below), so no chunk's memory is reused while its all-reduce runs - and no allocator
            # event is left pending on the comm stream (an allocation inside a later graph capture would
            # otherwise query it from the capturing thread)
            outs.append(y)
        self._ledger.join(cur, comm)
        return torch.cat(outs)

    def col_ok(self, lin) -> bool:
        """Can this row-parallel projection run column-chunked (_reduce_cols)?"""
        C = self.col_chunks
        return (self.tp.comm_active and C > 1 and not lin.glu and lin.N % (8 * C) == 0)

    def _reduce_cols(self, lin, x, pre=None) -> torch.Tensor:
        """``all_reduce(lin(pre(x) if pre else x))`` as C column chunks (the "col" decode schedule): chunk c is the
        GEMM over output features [c N/C, (c + 1) N/C) - a disjoint slice of the weight rows, so every weight byte is
        read once - into its own contiguous [M, N/C] block of a chunk-major [C, M, N/C] buffer, and its all-reduce
        is issued on the comm stream at once, while the compute stream already runs chunk c + 1's GEMM.
        The compute stream waits for the comm stream once, after the last chunk; add_norm reads the chunk-major
        layout directly. Reference: the synchronous row-parallel all-reduce, ``layers.py:175-179``."""
        h = pre(x) if pre is not None else x
        C, N = self.col_chunks, lin.N
        cw = N // C
        M = h.shape[0]
        out = torch.empty(C, M, cw, dtype=h.dtype, device=h.device)
        if not h.is_cuda:  # gloo / CPU: same chunks, collectives and ledger, no streams
            for c in range(C):
                out[c].copy_(lin.rows(c * cw, (c + 1) * cw)(h))
                self._ledger.fork(None, None)
                self.tp.all_reduce(out[c])
            self._ledger.join(None, None)
            return out
        cur = torch.cuda.current_stream()
        comm = self._comm(h.device)
        H = _hip_ops()
        for c in range(C):
            sl = lin.rows(c * cw, (c + 1) * cw)
            H.linear(h, sl.w, sl.b, w_scale=sl.w_scale, out=out[c])
            self._ledger.fork(cur, comm)  # chunk c's GEMM done
            with torch.cuda.stream(comm):
                self.tp.all_reduce(out[c])
        self._ledger.join(cur, comm)
        return out

    # ------------------------------------------------------- two-micro-batch decode overlap
    def overlap_split(self, B: int) -> int:
        """Rows in the first micro-batch of a B-row decode step (0 = no split)."""
        if self.tbo_min <= 0 or B < max(2, self.tbo_min) or not self.tp.comm_active:
            return 0
        return (B // 2 + 7) // 8 * 8 if B >= 32 else B // 2

    def prefill_split(self, inp: StepInput) -> Optional[Tuple[int, int]]:
        """(sequence index j, token row h) splitting a prefill step into sequences [0, j) / [j, B) with about
        half the tokens each, or None (no split: small step, one sequence, or no communication)."""
        if inp.kind != "prefill" or inp.cu_host is None or self.tbo_prefill_min <= 0 or not self.tp.comm_active:
            return None
        cu = [int(c) for c in inp.cu_host]
        T = cu[-1]
        if len(cu) < 3 or T < self.tbo_prefill_min:
            return None
        j = min(range(1, len(cu) - 1), key=lambda i: abs(2 * cu[i] - T))
        return j, cu[j]

    def _sub_prefill(self, inp: StepInput, j: int, h: int) -> Tuple[StepInput, StepInput]:
        cu = inp.cu_seqlens
        lens = [int(b) - int(a) for a, b in zip(inp.cu_host[:-1], inp.cu_host[1:])]

        def part(r0, r1, c, ls):
            return StepInput("prefill", inp.input_ids[r0:r1], inp.positions[r0:r1], inp.slots[r0:r1], cu_seqlens=c,
                             max_seqlen=max(ls))
        return part(0, h, cu[:j + 1], lens[:j]), part(h, int(inp.cu_host[-1]), cu[j:] - h, lens[j:])

    def _sub_step(self, inp: StepInput, r0: int, r1: int, block_size: int) -> StepInput:
        splits = inp.decode_splits
        if splits is not None and inp.input_ids.is_cuda:
            splits = _hip_ops().decode_splits(r1 - r0, self.plan.nkv_l, inp.max_ctx, block_size)
        return StepInput("decode", inp.input_ids[r0:r1], inp.positions[r0:r1], inp.slots[r0:r1],
                         block_tables=inp.block_tables[r0:r1], ctx_lens=inp.ctx_lens[r0:r1], max_ctx=inp.max_ctx,
                         decode_splits=splits)

    def _hidden_states_overlap(self, inp: StepInput, kv_caches, h: int, subs=None) -> torch.Tensor:
        """Decode step (or prefill step: ``subs`` from _sub_prefill) as two micro-batches (rows [0, h) and
        [h, B)) interleaved layer by layer.

        Compute-stream order per layer: A.attn, B.attn, A.mlp, B.mlp. Each block's all-reduce goes
        to the comm stream and the compute stream waits for it (event) only right
        before that micro-batch's next use, i.e. after the other micro-batch's block has been
        queued. RCCL therefore runs while the matrix cores work on the other half of the batch,
        instead of in series with them; the price is reading each layer's weight shard twice.
        All ranks queue the collectives in the same order (A before B), as RCCL requires.
        """
        cfg, w = self.cfg, self.w
        eps, rms = cfg.norm_eps, self.rms
        B = inp.input_ids.shape[0]
        bs = kv_caches[0][0].shape[2]
        if subs is None:
            subs = (self._sub_step(inp, 0, h, bs), self._sub_step(inp, h, B, bs))
        rows = ((0, h), (h, B))
        on_gpu = inp.input_ids.is_cuda
        cur = torch.cuda.current_stream() if on_gpu else None
        comm = self._comm(inp.input_ids.device) if on_gpu else None

        ledger = self._ledger

        def reduce(t):  # all-reduce t on the comm stream; returns the mark to wait on before reading t
            tok = ledger.fork(cur, comm)
            with (torch.cuda.stream(comm) if on_gpu else contextlib.nullcontext()):
                self.tp.all_reduce(t)
                # no record_stream (see _reduce_rows): the compute stream waits for this mark before it reads t or
                # drops its last reference (the next layer's ready(), or the final joins)
                return ledger.mark(comm, tok)

        def ready(mark):
            ledger.wait(cur, mark)

        x = ops.embed(inp.input_ids, w.wte, inp.positions if w.wpe is not None else None, w.wpe)
        delta = [x[r0:r1] for r0, r1 in rows]
        res: List[Optional[torch.Tensor]] = [None, None]
        pend = [None, None]
        for i, L in enumerate(w.layers):
            kc, vc = kv_caches[i]
            if cfg.parallel_block:  # GPT-J: one all-reduce per layer and micro-batch
                for j in (0, 1):
                    ready(pend[j])
                    y, res[j] = ops.add_norm(delta[j], L.ln1_w, L.ln1_b, eps, rms, res[j])
                    a = self._attention(L, y, subs[j], kc, vc)
                    delta[j] = L.o(a).add_(self._mlp(L, y))
                    pend[j] = reduce(delta[j])
                continue
            o = [None, None]
            for j in (0, 1):
                ready(pend[j])
                y, res[j] = ops.add_norm(delta[j], L.ln1_w, L.ln1_b, eps, rms, res[j])
                a = self._attention(L, y, subs[j], kc, vc)
                o[j] = L.o(a)
                pend[j] = reduce(o[j])
            for j in (0, 1):
                ready(pend[j])
                y2, res[j] = ops.add_norm(o[j], L.ln2_w, L.ln2_b, eps, rms, res[j])
                delta[j] = self._mlp(L, y2)
                pend[j] = reduce(delta[j])
        out = torch.empty_like(x)
        for j, (r0, r1) in enumerate(rows):
            ready(pend[j])
            ops.add_norm(delta[j], w.lnf_w, w.lnf_b, eps, rms, res[j], out=out[r0:r1])
        return out

    def rsag_ok(self, M: int) -> bool:
        """Can an M-row decode step run the row-sharded (reduce-scatter / all-gather) schedule?"""
        return self.tp.comm_active and self.tp.size > 1 and M % self.tp.size == 0 and M >= self.tp.size

    def _hidden_states_rsag(self, inp: StepInput, kv_caches) -> torch.Tensor:
        """Decode step with the residual stream sharded by rows across the TP ranks.

        Per layer: the row-parallel partial output (o, or down(up(.))) is REDUCE-SCATTERED - this rank gets the
        sums of its M / tp rows - the residual add + norm runs on those rows only, and the normed rows are
        ALL-GATHERED as the next column-parallel GEMM's input. The bytes on the wire equal the all-reduce's (an
        RCCL ring all-reduce is a reduce-scatter followed by an all-gather), but the two add_norm launches of a
        layer touch 1 / tp of the rows, and the embedding rows / residual need no replication. Numerically it
        is the all-reduce schedule: every row's sum and norm are computed once, on the rank owning the row."""
        cfg, w, tp = self.cfg, self.w, self.tp
        eps, rms = cfg.norm_eps, self.rms
        x = ops.embed(inp.input_ids, w.wte, inp.positions if w.wpe is not None else None, w.wpe)
        m = x.shape[0] // tp.size
        delta = x[tp.rank * m:(tp.rank + 1) * m]
        residual = None
        for i, L in enumerate(w.layers):
            kc, vc = kv_caches[i]
            y_sh, residual = ops.add_norm(delta, L.ln1_w, L.ln1_b, eps, rms, residual)
            y = tp.all_gather_rows(y_sh)
            a = self._attention(L, y, inp, kc, vc)
            if cfg.parallel_block:  # GPT-J: one reduce-scatter for attention + MLP
                delta = tp.reduce_scatter_rows(L.o(a).add_(self._mlp(L, y)))
                continue
            o_sh = tp.reduce_scatter_rows(L.o(a))
            y2_sh, residual = ops.add_norm(o_sh, L.ln2_w, L.ln2_b, eps, rms, residual)
            delta = tp.reduce_scatter_rows(self._mlp(L, tp.all_gather_rows(y2_sh)))
        h_sh, _ = ops.add_norm(delta, w.lnf_w, w.lnf_b, eps, rms, residual)
        return tp.all_gather_rows(h_sh)

    def hidden_states(self, inp: StepInput, kv_caches) -> torch.Tensor:
        h = self._hidden_states(inp, kv_caches)
        self._ledger.check("DecoderLM.hidden_states")  # every comm-stream fork joined (graph capture needs it)
        return h

    def _hidden_states(self, inp: StepInput, kv_caches) -> torch.Tensor:
        if inp.kind == "decode":
            B = inp.input_ids.shape[0]
            if self.rsag_ok(B) and (self.rsag_mode == "1" or B in self.rsag):
                return self._hidden_states_rsag(inp, kv_caches)
            h = self.overlap_split(B)
            if h:
                return self._hidden_states_overlap(inp, kv_caches, h)
        elif inp.kind == "prefill":
            sp = self.prefill_split(inp)
            if sp is not None:
                return self._hidden_states_overlap(inp, kv_caches, sp[1], subs=self._sub_prefill(inp, *sp))
        cfg, w = self.cfg, self.w
        eps, rms = cfg.norm_eps, self.rms
        x = ops.embed(inp.input_ids, w.wte, inp.positions if w.wpe is not None else None, w.wpe)
        residual = None
        delta = x
        fuse = self.tp.size == 1  # split-K partials can skip their own reduce only without a TP all-reduce
        col = (inp.kind == "decode" and not cfg.parallel_block and self.col_ok(w.layers[0].o)
               and self.col_ok(w.layers[0].down) and (self.col_mode == "force" or inp.input_ids.shape[0] in self.col))
        for i, L in enumerate(w.layers):
            kc, vc = kv_caches[i]
            y, residual = ops.add_norm(delta, L.ln1_w, L.ln1_b, eps, rms, residual, fp8_out=self._fp8_in(L.qkv, delta))
            # column-parallel QKV: its split-K partials are summed inside the rope/cache kernel
            a = self._attention(L, y, inp, kc, vc)
            if cfg.parallel_block:  # GPT-J: one all-reduce for attention + MLP
                delta = self._reduce_rows(lambda a_, y_: L.o(a_).add_(self._mlp(L, y_)), a, y)
            elif col:  # column-chunked all-reduces overlapping the next chunk's GEMM (_reduce_cols)
                o = self._reduce_cols(L.o, a)
                y2, residual = ops.add_norm(o, L.ln2_w, L.ln2_b, eps, rms, residual, fp8_out=self._fp8_in(L.up, a))
                delta = self._reduce_cols(L.down, y2, pre=lambda y_: L.up(y_, self.act))
            elif fuse:
                # TP=1: the split-K partials of o / down are reduced inside the next add_norm
                o = L.o(a, partial_ok=True)
                y2, residual = ops.add_norm(o, L.ln2_w, L.ln2_b, eps, rms, residual, fp8_out=self._fp8_in(L.up, a))
                delta = self._mlp(L, y2, partial_ok=True)
            else:
                o = self._reduce_rows(L.o, a)
                y2, residual = ops.add_norm(o, L.ln2_w, L.ln2_b, eps, rms, residual, fp8_out=self._fp8_in(L.up, a))
                delta = self._reduce_rows(lambda y_: self._mlp(L, y_), y2)
        h, _ = ops.add_norm(delta, w.lnf_w, w.lnf_b, eps, rms, residual)
        return h

    @property
    def vocab_lo(self) -> int:
        """Global token id of this rank's first LM-head row (vocab-parallel shard)."""
        return self.plan.rank * self.plan.v_l

    def local_logits(self, h: torch.Tensor) -> torch.Tensor:
        """[B, H] -> this rank's [B, Vpadded / tp] logit shard (no gather)."""
        return self.w.head(h)

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
