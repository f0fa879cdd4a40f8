"""Continuous-batching generation engine (one instance per tensor-parallel rank).

Reference counterpart: the decode loops inlined in ``generate.py:99-190`` and
``consumer_server.py:114-166`` - one batch at a time, KV cache grown with ``torch.cat``,
sampling on rank 0 followed by a ``dist.broadcast`` of the token every step, a host sync per
token and (no-cache mode) ``torch.cuda.empty_cache()`` per token.

Here:
* the C++ :class:`Scheduler` spends a per-step token budget on every running sequence's next
  token, then on prompt chunks (chunked prefill: a long prompt is split over steps and mixed with
  the running decodes, its chunks attending their cached prefix through the paged cache), then on
  FCFS admission (continuous batching, preemption by recompute);
* the KV cache is a preallocated paged pool sized from free HBM (288 GB per MI355X);
* decode steps replay a HIP graph captured per batch-size bucket (embedding -> all layers incl.
  RCCL all-reduces -> LM head -> all-gather -> sampler), so a step is one graph launch;
* every rank runs the same scheduler on the same request stream and samples the same token
  from the same all-gathered logits with the same per-step Philox key - no token broadcast.
"""
from __future__ import annotations

import collections
import contextlib
import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .. import _native, ops
from ..models.decoder import DecoderLM, StepInput
from ..ops import hip as _hip_ops
from ..utils.logging import get_logger
from ..utils.tracing import PhaseTimer
from ..utils.tracing import range as trace_range
from .sampling import SamplingParams, step_seeds

log = get_logger(__name__)

# context length (cached positions per row) at which the capture-time A/Bs time their candidates - the GQA decode
# attention kernels and the decode schedules: the bench's mean over a 128-token prompt + 128 generated tokens
AB_CTX = 192


@dataclass
class Request:
    id: int
    prompt_ids: List[int]
    params: SamplingParams
    seed: int
    output_ids: List[int] = field(default_factory=list)
    finished: bool = False
    finish_reason: str = ""
    t_arrival: float = 0.0
    t_first: float = 0.0
    t_last: float = 0.0
    token_times: List[float] = field(default_factory=list)

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def last_id(self) -> int:
        return self.output_ids[-1] if self.output_ids else self.prompt_ids[-1]

    def metrics(self) -> Dict[str, float]:
        ttft = self.t_first - self.t_arrival if self.t_first else float("nan")
        n = len(self.output_ids)
        tpot = (self.t_last - self.t_first) / (n - 1) if n > 1 else float("nan")
        return {"ttft_s": ttft, "tpot_s": tpot, "e2e_s": self.t_last - self.t_arrival, "output_tokens": n}


@dataclass
class StepEvent:
    req_id: int
    token: int
    finished: bool
    finish_reason: str = ""


class _DecodeBuffers:
    """Static device buffers feeding the captured decode graphs, filled by ONE host-to-device copy
    per step from one of two pinned staging sets: with decode steps pipelined (LLMEngine.step),
    the host fills step t+1's set while step t's copy may still be queued, so a set is rewritten
    only after the step that used it has been collected. Token ids come back through two pinned
    output buffers for the same reason."""

    def __init__(self, max_b: int, max_blocks: int, device):
        B, MB = max_b, max_blocks
        self.max_b, self.max_blocks = B, MB
        pin = torch.cuda.is_available() and device.type == "cuda"
        self.o32 = 4 * B * 8  # ids|pos|slots|seeds (i64) | ctx|topk|bt (i32) | temp|topp (f32)
        self.of32 = self.o32 + (2 * B + B * MB) * 4
        nbytes = self.of32 + 2 * B * 4
        self.h = [torch.zeros(nbytes, dtype=torch.uint8, pin_memory=pin) for _ in range(2)]
        self.d = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        self.d_i64 = self.d[:self.o32].view(torch.int64)
        self.d_i32 = self.d[self.o32:self.of32].view(torch.int32)
        self.d_f32 = self.d[self.of32:].view(torch.float32)
        self.out = torch.zeros(max_b, dtype=torch.int64, device=device)
        self.h_out = [torch.zeros(max_b, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self.ids, self.pos, self.slots, self.seeds = (self.d_i64[i * B:(i + 1) * B] for i in range(4))
        self.ctx, self.topk = self.d_i32[:B], self.d_i32[B:2 * B]
        self.bt = self.d_i32[2 * B:].view(B, max_blocks)
        self.temp, self.topp = self.d_f32[:B], self.d_f32[B:]

    def fill(self, k, b_pad, ids, pos, slots, seeds, ctx, topk, bt, temp, topp):
        """Stage one step's inputs in set k and copy them to the device. ``ids=None``: the input ids
        are the previous step's sampled tokens, copied on the device (same rows)."""
        n = len(pos)
        B, MB = self.max_b, self.max_blocks
        h = self.h[k]
        hi = h[:self.o32].view(torch.int64).numpy()
        hi32 = h[self.o32:self.of32].view(torch.int32).numpy()
        hf = h[self.of32:].view(torch.float32).numpy()
        for j, arr in enumerate((ids, pos, slots, seeds)):
            if arr is not None:
                hi[j * B:j * B + n] = arr
            hi[j * B + n:j * B + b_pad] = -1 if j == 2 else 0  # padded rows: no cache write
        hi32[:n] = ctx
        hi32[n:b_pad] = 0
        hi32[B:B + n] = topk
        hi32[B + n:B + b_pad] = 1
        btv = hi32[2 * B:].reshape(B, MB)
        btv[:n, :bt.shape[1]] = bt
        btv[n:b_pad] = 0
        hf[:n] = temp
        hf[n:b_pad] = 0
        hf[B:B + n] = topp
        hf[B + n:B + b_pad] = 1
        self.d.copy_(h, non_blocking=True)
        if ids is None:
            self.ids[:n].copy_(self.out[:n])


class LLMEngine:
    def __init__(self, model: DecoderLM, *, max_num_seqs: int = 256, max_batched_tokens: int = 8192,
                 block_size: int = 16, num_blocks: Optional[int] = None, max_model_len: Optional[int] = None,
                 kv_fraction: float = 0.9, use_graphs: Optional[bool] = None, eos_token_id: Optional[int] = None,
                 graph_buckets: Optional[Sequence[int]] = None, check_tokens: Optional[bool] = None,
                 autotune: Optional[bool] = None, prefill_chunk: Optional[int] = None,
                 kv_dtype: Optional[str] = None):
        self.model = model
        if kv_dtype is not None:  # "bf16" (model dtype) or "fp8" (e4m3 rows + per-row scale)
            if kv_dtype not in ("bf16", "fp8"):
                raise ValueError(f"kv_dtype must be 'bf16' or 'fp8', not {kv_dtype!r}")
            model.kv_fp8 = kv_dtype == "fp8"
        self.cfg = model.cfg
        self.tp = model.tp
        self.device = model.device
        self.is_gpu = self.device.type == "cuda"
        self.block_size = block_size
        self.max_model_len = min(max_model_len or self.cfg.max_position_embeddings, self.cfg.max_position_embeddings)
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max_batched_tokens
        self.eos = eos_token_id if eos_token_id is not None else self.cfg.eos_token_id
        self.max_blocks = math.ceil(self.max_model_len / block_size)
        # every rank runs its own scheduler on the same request stream, so the KV pool (admission,
        # preemption) must be identical everywhere: each rank sizes it from its own free HBM, then all
        # take the minimum
        self.num_blocks = self.tp.all_reduce_int(num_blocks or self._auto_blocks(kv_fraction), "min")
        self.kv = model.allocate_kv_cache(self.num_blocks, block_size)
        # chunked prefill: prompts are cut to fit the per-step token budget and ride along with the
        # running decodes (prefill_chunk > 0 caps a chunk further; < 0 keeps prompts whole)
        self.prefill_chunk = int(prefill_chunk if prefill_chunk is not None else
                                 os.environ.get("LLMSS_PREFILL_CHUNK", "0"))
        self.sched = _native().Scheduler(self.num_blocks, block_size, max_num_seqs, self.max_batched_tokens,
                                         self.max_model_len, self.prefill_chunk)
        self.requests: Dict[int, Request] = {}
        self._next_id = 0
        self._pending = collections.deque()  # launched GPU decode steps whose tokens are not yet processed
        self._last_rec = None  # last collected decode step (per-request constants for reuse)
        self._last_fins = None
        self._stage = 0  # pinned staging set of the next launch
        self._t_collect = 0.0  # when the last decode step was collected (non-overlapped decode_time_s)
        self._aborted = set()  # ids aborted while a decode step holding them was in flight
        self.async_decode = os.environ.get("LLMSS_ASYNC_DECODE", "1") != "0"
        self.check_tokens = check_tokens if check_tokens is not None else os.environ.get("LLMSS_CHECK_TOKENS") == "1"
        self.stats = {"steps": 0, "prefill_steps": 0, "decode_steps": 0, "tokens": 0, "prefill_tokens": 0,
                      "preemptions": 0, "decode_time_s": 0.0, "prefill_time_s": 0.0}
        self.timer = PhaseTimer()  # LLMSS_TIMING=1: HIP-event device time per phase; LLMSS_ROCTX=1: roctx ranges
        self._host_prof = self.timer.enabled  # LLMSS_TIMING=1 also records host-side time per engine phase
        self.use_graphs = self.is_gpu if use_graphs is None else (use_graphs and self.is_gpu)
        if self.tp.is_real and self.tp.host_staged:  # gloo-staged device collectives cannot be captured
            self.use_graphs = False
        self.graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}  # (batch bucket, candidate sampler) -> graph
        # vocab-parallel sampling from per-rank candidates (SURVEY R11 "better"): greedy / top-k <= 64 rows
        # gather [B, tp, 128] (value, id) pairs instead of [B, V] logits
        from ..ops.hip import CAND_KC, CAND_MAX_SHARD

        self.dist_sampling = (self.tp.size > 1
                              and self.tp.size * CAND_KC <= 2048  # sample_cand's gathered-candidate limit
                              and (not self.is_gpu or model.plan.v_l <= CAND_MAX_SHARD))
        self.buckets = sorted(set(graph_buckets or self._default_buckets()))
        self.buckets = [b for b in self.buckets if b <= max_num_seqs] or [max_num_seqs]
        if self.buckets[-1] < max_num_seqs:
            self.buckets.append(max_num_seqs)
        self._tbo_cands = self._tbo_candidates()
        self._rsag_cands = self._rsag_candidates()
        self._col_cands = self._col_candidates()
        # bucket -> decode schedule the capture-time A/B kept: "one" (all-reduce per row-parallel output),
        # "tbo" (two interleaved micro-batches), "rsag" (row-sharded: reduce-scatter / all-gather) or "col"
        # (column-chunked all-reduces beside the next chunk's GEMM)
        self.decode_schedule: Dict[int, str] = {}
        self.tp.check_consistent("LLMEngine", self.fingerprint())
        self.buf = _DecodeBuffers(self.buckets[-1], self.max_blocks, self.device) if self.is_gpu else None
        if self.is_gpu:
            _hip_ops.reserve_workspace(self.device, 64 << 20)
            for b in self.decode_batch_sizes():
                nsplit, _ = self._splits(b)
                if nsplit > 1:
                    _hip_ops._DECODE_WS.get(b, model.plan.nh_l, nsplit, self.cfg.head_dim, self.device)
        if autotune is None:
            autotune = os.environ.get("LLMSS_AUTOTUNE", "1") != "0"
        self.tuned = {}
        if self.is_gpu and autotune:  # per-shape GEMM plans for every decode bucket (ops/autotune.py)
            from ..ops.autotune import tune_model

            self.tuned = tune_model(model, self.decode_batch_sizes())
        if self.is_gpu and autotune:
            self._tune_gqa_attention()
        if self.use_graphs and os.environ.get("LLMSS_GRAPHS", "1") == "0":
            self.use_graphs = False
        self._capture_agreed()

    def _capture_agreed(self):
        """Capture the decode graphs, agreeing on the outcome across TP ranks: if capture fails on ANY rank
        (e.g. a collective backend that refuses stream capture), every rank drops its graphs and decodes
        eagerly - a rank deciding alone would replay graphs whose collectives its eager peer issues in a
        different order, or wait in the A/B below for a rank that never comes. Then the capture-time A/B of
        the two-micro-batch schedule (real communicator only), then a second consistency check whose
        fingerprint holds the graph set and the A/B's choice."""
        if self.use_graphs:
            def capture():
                if os.environ.get("LLMSS_FAULT_INJECT", "") == f"{self.tp.rank}:capture:raise":  # tests
                    raise RuntimeError("injected decode graph capture failure")
                self.capture_graphs()
            ok, err = self.tp.agree(capture)
            if not ok:
                log.warning("decode graph capture failed (%s): every rank decodes eagerly",
                            err or "on a peer rank")
                if self.is_gpu:
                    torch.cuda.synchronize()
                self.graphs.clear()
                self.use_graphs = False
            elif self._tbo_cands or self._rsag_cands or self._col_cands:
                self._schedule_ab(self._graph_pool, self._graph_modes)
        self.tp.check_consistent("LLMEngine (after graph capture)", self.fingerprint())

    # -------------------------------------------------------------------------- sizing
    def fingerprint(self) -> dict:
        """Everything that steers scheduling or the collective sequence; must match on all TP ranks."""
        cfg = self.cfg
        return {"model": repr(sorted((k, str(v)) for k, v in cfg.__dict__.items())),
                "dtype": str(self.model.dtype), "tp": self.tp.size, "block_size": self.block_size,
                "num_blocks": self.num_blocks, "max_model_len": self.max_model_len,
                "max_num_seqs": self.max_num_seqs, "max_batched_tokens": self.max_batched_tokens,
                "buckets": list(self.buckets), "graphs": bool(self.use_graphs),
                "async_decode": self.async_decode, "eos": self.eos, "prefill_chunk": self.prefill_chunk,
                "dist_sampling": self.dist_sampling, "kv_fp8": bool(self.model.kv_fp8),
                "overlap_rows": self.model.overlap_rows, "bucket_bytes": self.model.bucket_bytes,
                "tbo_min": self.model.tbo_min, "graph_keys": sorted(self.graphs),
                "decode_schedule": sorted(self.decode_schedule.items()), "rsag_mode": self.model.rsag_mode,
                "col": [self.model.col_mode, self.model.col_chunks, sorted(self.model.col)],
                "fp8": any(L.qkv.w_scale is not None for L in self.model.w.layers[:1])}

    def _default_buckets(self):
        out, b = [], 1
        while b < self.max_num_seqs:
            out.append(b)
            b = b * 2 if b < 8 else b + (8 if b < 64 else 32)
        out.append(self.max_num_seqs)
        return out

    def _auto_blocks(self, frac: float) -> int:
        per = self.model.kv_bytes_per_block(self.block_size)
        want = self.max_num_seqs * self.max_blocks + 1
        if self.is_gpu:
            free, _ = torch.cuda.mem_get_info(self.device)
            budget = int(free * frac) - (4 << 30)
            n = max(64, budget // per)
            return int(min(n, want))
        return int(min(want, max(64, (2 << 30) // per)))

    def decode_batch_sizes(self) -> List[int]:
        """Row counts the decode kernels run at: every bucket, plus both micro-batch halves of the
        buckets that DecoderLM splits for all-reduce / compute overlap (or that the capture-time A/B
        may split, _tbo_candidates)."""
        out = set(self.buckets)
        for b in self.buckets:
            h = self.model.overlap_split(b) or self._tbo_half(b)
            if h:
                out.update((h, b - h))
        return sorted(out)

    def _tune_gqa_attention(self):
        """For grouped-query models (>= 4 query heads per kv head, e.g. Llama-2-70B's 8, MQA's all) time the VALU
        split-K decode kernel against the MFMA extend kernel per decode bucket on a synthetic cache (context
        AB_CTX) and route the buckets where MFMA wins (DecoderLM.gqa_mfma). Every rank
        sees the same shapes; the decision is agreed through all_reduce_int so the ranks run the same kernels."""
        m, p, cfg = self.model, self.model.plan, self.cfg
        if p.nh_l // max(1, p.nkv_l) < 4:
            return
        from ..ops.autotune import _time

        D, dev = cfg.head_dim, self.device
        ctx = max(1, min(AB_CTX, self.max_model_len - 1))
        nblk = -(-ctx // self.block_size)
        res = {}
        for b in self.decode_batch_sizes():
            if b < 8:
                continue
            nb = b * nblk
            kc = torch.randn(nb, p.nkv_l, self.block_size, D, device=dev).to(m.dtype) if not m.kv_fp8 else None
            if kc is None:
                return
            vc = torch.randn_like(kc)
            qkv = torch.randn(b, (p.nh_l + 2 * p.nkv_l) * D, device=dev).to(m.dtype)
            bt = torch.arange(nb, dtype=torch.int32, device=dev).view(b, nblk)
            bt = torch.nn.functional.pad(bt, (0, self.max_blocks - nblk))
            cl = torch.full((b,), ctx, dtype=torch.int32, device=dev)
            out = torch.empty(b, p.nh_l * D, dtype=m.dtype, device=dev)
            cu = m.decode_cu(b, dev)
            sp = self._splits(b)

            def valu(i):
                ops.attn_decode(qkv, kc, vc, bt, cl, p.nh_l, p.nkv_l, D, m.scale, self.max_model_len, splits=sp,
                                out=out)

            def mfma(i):
                ops.attn_extend(qkv, kc, vc, bt, cu, cl, 1, p.nh_l, p.nkv_l, D, m.scale, out=out)
            valu(0)
            mfma(0)
            torch.cuda.synchronize()
            tv, tm = _time(valu, 8), _time(mfma, 8)
            win = self.tp.all_reduce_int(int(tm < 0.97 * tv), "min")
            if win:
                m.gqa_mfma.add(b)
            res[b] = (round(tv, 1), round(tm, 1))
            del kc, vc
        self.stats["gqa_attn_us"] = {str(b): v for b, v in res.items()}
        log.info("GQA decode attention (us VALU split-K / MFMA extend): %s; MFMA for %s", res, sorted(m.gqa_mfma))

    def _tbo_candidates(self) -> List[int]:
        """Decode buckets whose two-micro-batch schedule is timed against the single-batch one at capture
        only with a real multi-rank communicator - on one GPU there is nothing to overlap - and for buckets of
        >= LLMSS_TBO_AUTO_MIN (default 128; 0 = no micro-batch A/B) sequences."""
        if not (self.is_gpu and self.tp.is_real and not self.tp.host_staged and self.model.tbo_min <= 0
                and int(os.environ.get("LLMSS_TBO_AUTO_MIN", "128")) > 0):
            return []
        lo = int(os.environ.get("LLMSS_TBO_AUTO_MIN", "128"))
        return [b for b in self.buckets if b >= lo]

    def _rsag_candidates(self) -> List[int]:
        """Decode buckets whose row-sharded schedule (reduce-scatter -> add + norm on M / tp rows -> all-gather,
        DecoderLM._hidden_states_rsag) is timed against the all-reduce one at capture: real multi-rank
        communicator, LLMSS_TP_RSAG=auto (default), buckets divisible by the TP degree of at least
        8 rows per rank. Not for fp8-weight models: their default schedule feeds the
        GEMMs the fp8 twin that add_norm writes, which the row-sharded add + norm does not produce, so the A/B would
        not compare like with like."""
        m = self.model
        if not (self.is_gpu and self.tp.is_real and not self.tp.host_staged and m.rsag_mode == "auto"):
            return []
        if any(L.qkv.w_scale is not None for L in m.w.layers[:1]):
            return []
        lo = 8 * self.tp.size
        return [b for b in self.buckets if b >= lo and m.rsag_ok(b)]

    def _col_candidates(self) -> List[int]:
        """Decode buckets whose column-chunked schedule (DecoderLM._reduce_cols: each row-parallel projection as
        LLMSS_TP_COL chunks over disjoint weight-row slices, chunk c's all-reduce on the comm stream beside chunk
        c + 1's GEMM) is timed against the single all-reduce at capture: real multi-rank communicator, "auto" mode,
        sequential-block models whose o / down widths split into 8-aligned chunks."""
        m = self.model
        if not (self.is_gpu and self.tp.is_real and not self.tp.host_staged and m.col_mode == "auto"):
            return []
        L = m.w.layers[0]
        if self.cfg.parallel_block or not (m.col_ok(L.o) and m.col_ok(L.down)):
            return []
        return [b for b in self.buckets if b >= m.col_min]

    def _tbo_half(self, b: int) -> int:
        if b not in getattr(self, "_tbo_cands", ()):
            return 0
        m = self.model
        old, m.tbo_min = m.tbo_min, b
        try:
            return m.overlap_split(b)
        finally:
            m.tbo_min = old

    def _splits(self, b):
        return _hip_ops.decode_splits(b, self.model.plan.nkv_l, self.max_model_len, self.block_size)

    # -------------------------------------------------------------------------- requests
    def add_request(self, prompt_ids: Sequence[int], params: Optional[SamplingParams] = None,
                    req_id: Optional[int] = None) -> int:
        params = params or SamplingParams()
        prompt = list(int(t) for t in prompt_ids)
        if not prompt:
            raise ValueError("empty prompt")
        max_new = min(params.max_new_tokens, self.max_model_len - 1)
        if len(prompt) + max_new > self.max_model_len:  # left-truncate like the reference tokenizer
            prompt = prompt[-(self.max_model_len - max_new):]
        if params.max_new_tokens != max_new:
            params = SamplingParams(**{**params.__dict__, "max_new_tokens": max_new})
        rid = self._next_id if req_id is None else int(req_id)
        self._next_id = max(self._next_id, rid + 1)
        req = Request(rid, prompt, params, params.resolved_seed(), t_arrival=time.perf_counter())
        # the scheduler validates first (a sequence larger than the whole KV pool, a whole prompt over the token
        # budget -> ValueError): a rejected request is never registered, so nothing is left behind
        self.sched.add(rid, len(prompt), max_new)
        self.requests[rid] = req
        return rid

    def abort(self, rid: int):
        if rid in self.requests:
            self.sched.abort(rid)
            r = self.requests[rid]
            r.finished, r.finish_reason = True, "abort"
            if self._pending:  # rows of in-flight decode steps: no speculative successor may touch it
                self._aborted.add(rid)

    def has_unfinished(self) -> bool:
        return self.sched.has_work() or bool(self._pending)

    def pop_finished(self) -> List[Request]:
        done = [r for r in self.requests.values() if r.finished]
        for r in done:
            del self.requests[r.id]
            self._aborted.discard(r.id)
        return done

    # -------------------------------------------------------------------------- step
    def _sampling_arrays(self, reqs: List[Request]):
        temp = np.array([r.params.k_temperature for r in reqs], dtype=np.float32)
        topk = np.array([r.params.k_top_k for r in reqs], dtype=np.int32)
        topp = np.array([r.params.k_top_p for r in reqs], dtype=np.float32)
        seeds = step_seeds(np.array([r.seed for r in reqs], dtype=np.uint64),
                           np.array([len(r.output_ids) for r in reqs], dtype=np.int64))
        return temp, topk, topp, seeds

    def step(self) -> List[StepEvent]:
        """One engine iteration; returns the token events it completed.

        GPU decode steps are pipelined with the host. While the running set only advances (no
        waiting prompt, no sequence entering a new KV block) the NEXT decode step is launched
        before the current one is collected: its input ids are the current step's sampled
        tokens, copied on the device, and its positions / slots / context lengths / Philox keys
        are the current ones + 1, so the GPU never waits for Python bookkeeping. A sequence
        that stops on EOS / a stop token in step t has computed one extra token in step t+1,
        which is dropped. Otherwise (prefill admission, a block boundary, preemption) the
        scheduler runs between the two steps as usual.
        """
        hp = self._host_prof
        t_a = time.perf_counter() if hp else 0.0
        done = None
        if self._pending:
            if self.async_decode and self.sched.num_waiting() == 0 and self.sched.num_prefilling() == 0:
                self._speculate(self._pending[-1])
            done = self._collect_decode()
            if self._pending:  # the next step is already in flight
                if hp:
                    self.stats["host_collect_apply_s"] = self.stats.get("host_collect_apply_s", 0.0) + \
                        time.perf_counter() - t_a
                return self._emit(*done)
        t_b = time.perf_counter() if hp else 0.0
        with trace_range("schedule"):
            batch = self.sched.schedule()
        if hp:
            t_c = time.perf_counter()
            self.stats["host_collect_apply_s"] = self.stats.get("host_collect_apply_s", 0.0) + t_b - t_a
            self.stats["host_schedule_s"] = self.stats.get("host_schedule_s", 0.0) + t_c - t_b
        new_events: List[StepEvent] = []
        if batch.kind == 0 and done is None and self.sched.has_work():
            # the scheduler preempts its way out of a starved pool, so an idle step with work left is a bug
            raise RuntimeError(f"scheduler returned an idle step with {self.sched.num_waiting()} waiting and "
                               f"{self.sched.num_running()} running sequences")
        if batch.kind != 0:
            self.stats["preemptions"] += len(batch.preempted)
            ids = batch.ids
            reqs = [self.requests[i] for i in ids.tolist()]
            if batch.kind == 1:  # prompt chunks (possibly with decode tokens riding along)
                t0 = time.perf_counter()
                with self.timer.phase("prefill"):
                    tokens = self._extend(batch, reqs)
                self.stats["prefill_steps"] += 1
                self.stats["prefill_tokens"] += int(batch.query_lens[batch.num_decode:].sum())
                self.stats["mixed_decode_tokens"] = self.stats.get("mixed_decode_tokens", 0) + batch.num_decode
                self.stats["prefill_time_s"] += time.perf_counter() - t0
                smp = batch.sample
                new_events = self._emit(*self._apply(ids[smp], [r for r, f in zip(reqs, smp) if f], tokens))
            elif self.is_gpu:
                self._launch_decode(self._record_from_batch(batch, ids, reqs))
            else:
                t0 = time.perf_counter()
                tokens = self._decode_cpu(batch, reqs)
                self.stats["decode_steps"] += 1
                self.stats["decode_time_s"] += time.perf_counter() - t0
                new_events = self._emit(*self._apply(ids, reqs, tokens))
        if hp:
            t_d = time.perf_counter()
            self.stats["host_launch_s"] = self.stats.get("host_launch_s", 0.0) + t_d - t_c
        events = (self._emit(*done) if done is not None else []) + new_events
        if hp:
            self.stats["host_emit_s"] = self.stats.get("host_emit_s", 0.0) + time.perf_counter() - t_d
        return events

    def _apply(self, ids: np.ndarray, reqs: List[Request], tokens: List[int]):
        """Critical-path bookkeeping of one step's tokens: append, stop checks, scheduler update."""
        if self.check_tokens and self.tp.is_real:
            allt = self.tp.all_gather_object(tokens)
            if any(t != tokens for t in allt):
                raise RuntimeError(f"rank {self.tp.rank}: sampled tokens diverged across TP ranks: {allt}")
        eos = self.eos
        reasons = [""] * len(reqs)
        fins = np.zeros(len(reqs), dtype=bool)
        for i, (r, tok) in enumerate(zip(reqs, tokens)):
            out = r.output_ids
            out.append(tok)
            p = r.params
            if len(out) >= p.max_new_tokens:
                reasons[i] = "length"
            elif not p.ignore_eos and eos is not None and tok == eos:
                reasons[i] = "eos"
            elif p.stop_token_ids and tok in p.stop_token_ids:
                reasons[i] = "stop"
            else:
                continue
            fins[i] = True
        self.sched.on_tokens(ids, fins)
        self._last_fins = fins
        self.stats["steps"] += 1
        return reqs, tokens, reasons, time.perf_counter()

    def _emit(self, reqs, tokens, reasons, now) -> List[StepEvent]:
        events = []
        for r, tok, reason in zip(reqs, tokens, reasons):
            if not r.t_first:
                r.t_first = now
            r.t_last = now
            r.token_times.append(now)
            if reason:
                r.finished, r.finish_reason = True, reason
            events.append(StepEvent(r.id, tok, bool(reason), reason))
        self.stats["tokens"] += len(events)
        return events

    def _extend(self, batch, reqs: List[Request]) -> List[int]:
        """A step with prompt chunks: rows [0, num_decode) are decode tokens, then one chunk per
        prompting sequence (positions ctx - q .. ctx - 1). Returns the tokens sampled for the
        sequences whose known tokens the step completes (batch.sample)."""
        dev = self.device
        qlens = batch.query_lens.astype(np.int64)
        ctx = batch.ctx_lens.astype(np.int64)
        nd = int(batch.num_decode)
        ids = np.concatenate([np.asarray(r.all_ids[c - q:c], dtype=np.int64) for r, q, c in zip(reqs, qlens, ctx)])
        ends = np.cumsum(qlens)
        cu = np.zeros(len(reqs) - nd + 1, dtype=np.int32)
        cu[1:] = ends[nd:] - (ends[nd - 1] if nd else 0)
        smp = batch.sample
        has_prefix = bool((ctx[nd:] > qlens[nd:]).any())
        kind = "prefill" if nd == 0 and not has_prefix else "extend"

        def d(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=True)

        inp = StepInput(
            kind=kind, input_ids=d(ids), positions=d(batch.positions), slots=d(batch.slots), cu_seqlens=d(cu),
            max_seqlen=int(qlens[nd:].max()), last_idx=d((ends - 1)[smp]),
            block_tables=d(batch.block_table.astype(np.int32)) if kind == "extend" else None,
            ctx_lens=d(ctx.astype(np.int32)) if kind == "extend" else None, max_ctx=self.max_model_len,
            num_decode=nd, has_prefix=has_prefix, cu_host=cu if kind == "prefill" else None)
        reqs = [r for r, f in zip(reqs, smp) if f]
        if not reqs:
            self.model.hidden_states(inp, self.kv)  # prompt chunks only: fill the cache, nothing to sample
            return []
        temp, topk, topp, seeds = self._sampling_arrays(reqs)
        tok = self._forward_sample(inp, *(torch.from_numpy(a).to(dev) for a in (temp, topk, topp, seeds)),
                                   dist=self._dist_ok(temp, topk))
        return tok.cpu().tolist()

    def _dist_ok(self, temp, topk) -> bool:
        """Sample this step from vocab-parallel candidates (no [B, V] logits all-gather)?"""
        return self.dist_sampling and ops.cand_ok(temp, topk)

    def _forward_sample(self, inp: StepInput, temp, topk, topp, seeds, out=None, dist=False):
        """Forward + LM head + sampler. ``dist``: each rank keeps its logit shard and only candidates
        are gathered (ops.sample_distributed); otherwise the [B, V] logits are all-gathered."""
        m = self.model
        V = self.cfg.vocab_size
        if dist:
            h = m.hidden_states(inp, self.kv)
            if inp.last_idx is not None:
                h = h.index_select(0, inp.last_idx)
            return ops.sample_distributed(m.local_logits(h), self.tp, m.vocab_lo, V, temp, topk, topp, seeds, out=out)
        logits = m(inp, self.kv)
        if logits.is_cuda:
            return _hip_ops.sample(logits, temp, topk, topp, seeds, vocab=min(V, logits.shape[-1]), out=out)
        return ops.sample(logits, temp, topk, topp, seeds, vocab=min(V, logits.shape[-1]))

    def _decode_forward(self, b: int, buf: _DecodeBuffers, dist: bool = False):
        inp = StepInput(kind="decode", input_ids=buf.ids[:b], positions=buf.pos[:b], slots=buf.slots[:b],
                        block_tables=buf.bt[:b], ctx_lens=buf.ctx[:b], max_ctx=self.max_model_len,
                        decode_splits=self._splits(b))
        self._forward_sample(inp, buf.temp[:b], buf.topk[:b], buf.topp[:b], buf.seeds[:b], out=buf.out[:b],
                             dist=dist)

    def _decode_cpu(self, batch, reqs: List[Request]) -> List[int]:
        ids = np.array([r.last_id for r in reqs], dtype=np.int64)
        temp, topk, topp, seeds = self._sampling_arrays(reqs)
        inp = StepInput(kind="decode", input_ids=torch.from_numpy(ids), positions=torch.from_numpy(batch.positions),
                        slots=torch.from_numpy(batch.slots),
                        block_tables=torch.from_numpy(batch.block_table.astype(np.int32)),
                        ctx_lens=torch.from_numpy(batch.ctx_lens.astype(np.int32)), max_ctx=self.max_model_len)
        return self._forward_sample(inp, temp, topk, topp, seeds, dist=self._dist_ok(temp, topk)).tolist()

    # ------------------------------------------------------------------ pipelined GPU decode
    def _record_from_batch(self, batch, ids: np.ndarray, reqs: List[Request]) -> dict:
        """Decode step record for a scheduled batch. Per-request constants are reused from the last
        collected step when the running set is unchanged (every member then got one token)."""
        last = self._last_rec
        if last is not None and last["ids"].shape == ids.shape and np.array_equal(last["ids"], ids) \
                and last["keep"].all():
            c = {k: last[k] for k in ("temp", "topk", "topp", "seed", "maxnew")}
            c["nout"] = last["nout"] + 1
            c["last"] = last["tokens"]
        else:
            c = {"temp": np.array([r.params.k_temperature for r in reqs], dtype=np.float32),
                 "topk": np.array([r.params.k_top_k for r in reqs], dtype=np.int32),
                 "topp": np.array([r.params.k_top_p for r in reqs], dtype=np.float32),
                 "seed": np.array([r.seed for r in reqs], dtype=np.uint64),
                 "maxnew": np.array([r.params.max_new_tokens for r in reqs], dtype=np.int64),
                 "nout": np.array([len(r.output_ids) for r in reqs], dtype=np.int64),
                 "last": np.array([r.last_id for r in reqs], dtype=np.int64)}
        c.update(ids=ids, reqs=reqs, n=len(reqs), pos=batch.positions, ctx=batch.ctx_lens.astype(np.int32),
                 slots=batch.slots, bt=batch.block_table, keep=np.ones(len(reqs), dtype=bool))
        c["dist"] = self._dist_ok(c["temp"], c["topk"])
        return c

    def _launch_decode(self, rec: dict, device_ids: bool = False):
        n = rec["n"]
        rec["t0"] = time.perf_counter()
        b = next(x for x in self.buckets if x >= n)
        k = self._stage
        self._stage ^= 1
        buf = self.buf
        with self.timer.phase("decode"):
            buf.fill(k, b, None if device_ids else rec.pop("last"), rec["pos"], rec["slots"],
                     step_seeds(rec["seed"], rec["nout"]), rec["ctx"], rec["topk"], rec["bt"], rec["temp"],
                     rec["topp"])
            key = (b, bool(rec["dist"]))
            if self._host_prof:
                # was the GPU already idle (every earlier step done) when this step was launched?
                idle = bool(self._pending) and self._pending[-1]["ev"].query()
                self.stats["host_late_launches"] = self.stats.get("host_late_launches", 0) + int(idle)
                t_r = time.perf_counter()
            if self.use_graphs and key in self.graphs:
                self.graphs[key].replay()
            else:
                self._decode_forward(b, buf, dist=key[1])
            if self._host_prof:
                self.stats["host_replay_s"] = self.stats.get("host_replay_s", 0.0) + time.perf_counter() - t_r
            buf.h_out[k][:n].copy_(buf.out[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        rec.update(k=k, ev=ev)
        self._pending.append(rec)

    def _speculate(self, cur: dict):
        """Launch the step after ``cur`` (still in flight) if it needs no scheduler decision."""
        alive = cur["keep"] & (cur["nout"] + 1 < cur["maxnew"])
        if self._aborted:
            # aborted while in flight: the scheduler has already released the sequence (no block to reserve,
            # no on_tokens); the row rides along as padding and is dropped at collect time
            alive &= ~np.isin(cur["ids"], np.fromiter(self._aborted, dtype=np.int64))
        if not alive.any():
            return
        nxt_pos = cur["pos"] + 1
        slots = np.where(alive, cur["slots"] + 1, -1)
        bt = cur["bt"]
        cross = np.flatnonzero(alive & (nxt_pos % self.block_size == 0))
        if cross.size:
            # sequences entering a new KV block get it now (Scheduler.reserve; the next schedule() finds it
            # allocated), so the pipeline does not drain every block_size steps; an empty pool leaves the step
            # to the scheduler, which may preempt
            bt = bt.copy()
            bs = self.block_size
            for i in cross:
                blk = self.sched.reserve(int(cur["ids"][i]), int(nxt_pos[i]) + 1)
                if blk < 0:
                    return
                bt[i, int(nxt_pos[i]) // bs] = blk
                slots[i] = blk * bs
            self.stats["spec_block_reserves"] = self.stats.get("spec_block_reserves", 0) + int(cross.size)
        dead = ~alive
        rec = {k: cur[k] for k in ("ids", "reqs", "n", "temp", "topk", "topp", "seed", "maxnew", "dist")}
        rec["bt"] = bt
        rec["pos"] = nxt_pos
        rec["ctx"] = np.where(alive, cur["ctx"] + 1, 0).astype(np.int32)
        rec["slots"] = slots
        rec["nout"] = cur["nout"] + 1
        rec["keep"] = alive
        if dead.any():
            rec["topk"] = np.where(alive, cur["topk"], 1).astype(np.int32)
        self._launch_decode(rec, device_ids=True)

    def _collect_decode(self):
        rec = self._pending.popleft()
        ev = rec["ev"]
        if self._host_prof:
            t = time.perf_counter()
            ev.synchronize()
            self.stats["host_gpu_wait_s"] = self.stats.get("host_gpu_wait_s", 0.0) + time.perf_counter() - t
        else:
            ev.synchronize()
        toks = self.buf.h_out[rec["k"]][:rec["n"]].numpy().copy()
        reqs = rec["reqs"]
        keep = rec["keep"]
        gone = [i for i in np.flatnonzero(keep) if reqs[i].finished]  # aborted while in flight
        if gone:
            keep = keep.copy()
            keep[gone] = False
            rec["keep"] = keep
        rows = np.flatnonzero(keep)
        ids = rec["ids"][rows]
        sel = [reqs[i] for i in rows]
        tokens = toks[rows].tolist()
        self.stats["decode_steps"] += 1
        # wall time without overlap: pipelined steps are in flight together, so each collected step counts from
        # its launch or from the previous collection, whichever is later
        now = time.perf_counter()
        self.stats["decode_time_s"] += now - max(rec["t0"], self._t_collect)
        self._t_collect = now
        out = self._apply(ids, sel, tokens)
        fins = self._last_fins
        nxt = self._pending[0] if self._pending else None
        if nxt is not None:  # the speculated successor drops rows that stopped (eos / stop / abort) here
            nk = nxt["keep"] & keep
            nk[rows[fins]] = False
            nxt["keep"] = nk
        rec["tokens"] = toks
        self._last_rec = rec
        return out

    def phase_summary(self) -> Dict[str, Dict[str, float]]:
        """Per-phase device time (LLMSS_TIMING=1) - {"prefill": {...}, "decode": {...}}."""
        return self.timer.summary()

    # -------------------------------------------------------------------------- graphs
    def capture_graphs(self):
        """Capture one decode graph per batch bucket (largest first, shared memory pool)."""
        buf = self.buf
        pool = torch.cuda.graph_pool_handle()
        # padded rows are harmless: ctx 0 -> zero attention, slot -1 -> no cache write
        buf.d_i64.zero_()
        buf.slots.fill_(-1)
        buf.d_i32.zero_()
        buf.topk.fill_(1)
        buf.d_f32.zero_()
        modes = self._decode_modes()
        # warm-up passes (lazy allocations, first launches). Native RCCL: with real collectives, so each
        # algorithm's lazy peer connection happens here and not inside the capture. torch's RCCL process
        # group: collectives suspended - its watchdog thread would otherwise still track the warm-up's work
        # items when the capture starts, and a watchdog query of their end events (recorded on the
        # communicator's stream, which the captured collectives pull into the capture) aborts the process
        torch_pg = self.tp.is_real and self.tp.comm is None and not self.tp.host_staged
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), (self.tp.suspended() if torch_pg else contextlib.nullcontext()):
            for b in reversed(self.buckets):
                for d in modes:
                    for _ in range(2):
                        self._decode_forward(b, buf, dist=d)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # settle the caching allocator's pending cross-stream events (freed side-stream blocks) outside the
        # capture, so no allocation during capture queries an event
        torch.cuda.empty_cache()
        # thread-local capture: the RCCL communicator's watchdog thread keeps querying the events of earlier
        # collectives; under the default global capture mode such a query from another thread aborts the
        # process ("operation not permitted when stream is capturing")
        for b in reversed(self.buckets):
            for d in modes:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                    self._decode_forward(b, buf, dist=d)
                self.graphs[(b, d)] = g
        torch.cuda.synchronize()
        self._graph_pool, self._graph_modes = pool, modes  # for the capture-time A/B (_capture_agreed)
        log.info("captured %d decode graphs: buckets %s, samplers %s", len(self.graphs), self.buckets,
                 ["candidates" if d else "gathered" for d in modes])

    def _decode_modes(self):
        """Sampler modes a decode graph is captured for: vocab-parallel runs get both samplers (candidates when every
        row allows it, else the gathered-logits sampler), chosen per step."""
        return (True, False) if self.dist_sampling else (False,)

    @contextlib.contextmanager
    def _schedule(self, b: int, name: str):
        """Decode bucket ``b`` runs schedule ``name`` inside the block (capture / warm-up of an A/B variant)."""
        m = self.model
        old_tbo, had, had_col = m.tbo_min, b in m.rsag, b in m.col
        if name == "tbo":
            m.tbo_min = b
        elif name == "rsag":
            m.rsag.add(b)
        elif name == "col":
            m.col.add(b)
        try:
            yield
        finally:
            m.tbo_min = old_tbo
            if name == "rsag" and not had:
                m.rsag.discard(b)
            if name == "col" and not had_col:
                m.col.discard(b)

    @staticmethod
    def _ab_buckets(cands: List[int]) -> List[int]:
        """The buckets the schedule A/B times: the largest candidate, the largest one at most half of it and the
        smallest one; every other candidate bucket adopts the winner of the nearest timed bucket (engine start-up at
        TP=8: 3 timed buckets instead of up to 15)."""
        cands = sorted(cands)
        if not cands:
            return []
        top = cands[-1]
        half = [b for b in cands if b <= top // 2]
        return sorted({top, cands[0]} | ({half[-1]} if half else set()))

    def _schedule_ab(self, pool, modes):
        """Capture-time A/B of the decode schedules on the real communicator: per timed bucket the
        all-reduce graph ("one") against the two-micro-batch one ("tbo": each half's all-reduces on the comm
        stream while the other half computes, DecoderLM._hidden_states_overlap), the row-sharded one ("rsag":
        reduce-scatter, add + norm on M / tp rows, all-gather, DecoderLM._hidden_states_rsag) and, when enabled, the
        column-chunked one ("col": each row-parallel output as C weight-row slices whose all-reduces run beside the
        next slice's GEMM, DecoderLM._reduce_cols). Each graph is replayed with a realistic context length (the
        bench's 128 + 64 average), every rank's times are gathered and the max over ranks decides, so all ranks keep
        the same graph; an alternative must beat "one" by 3 %. The other candidate buckets then capture the winner
        of their nearest timed bucket (_ab_buckets). Which wins depends on what collectives cost on the node - hence
        measured, not assumed (the split loses on one GPU: half-batch kernels are nearly as long as full ones,
        profiles/r1_tbo)."""
        buf, m = self.buf, self.model
        ctx = max(1, min(AB_CTX, self.max_model_len - 1))
        nblk = -(-ctx // self.block_size)
        if nblk > self.num_blocks:
            return
        variants = {b: [n for n, c in (("tbo", self._tbo_cands), ("rsag", self._rsag_cands), ("col", self._col_cands))
                        if b in c]
                    for b in self.buckets}
        variants = {b: v for b, v in variants.items() if v}
        timed_b = self._ab_buckets(list(variants))
        alt, times = {}, {}

        def forwards(pairs, suspended):  # eager forward of each (bucket, schedule) on a side stream
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), (self.tp.suspended() if suspended else contextlib.nullcontext()):
                for b, name in pairs:
                    with self._schedule(b, name):
                        self._decode_forward(b, buf, dist=modes[0])
            torch.cuda.current_stream().wait_stream(st)
            torch.cuda.synchronize()

        def capture_all(triples):
            for b, d, name in triples:
                with self._schedule(b, name):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                        self._decode_forward(b, buf, dist=d)
                alt[(b, d, name)] = g
            torch.cuda.synchronize()

        def timed(g):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                g.replay()
            e.record()
            e.synchronize()
            return s.elapsed_time(e) / 3

        def measure():
            # realistic rows for timing: every row attends `ctx` cached positions (garbage K/V, no cache writes)
            buf.ctx.fill_(ctx)
            buf.bt.zero_()
            buf.bt[:, :nblk] = torch.arange(nblk, dtype=torch.int32, device=buf.bt.device)
            for b in sorted(timed_b, reverse=True):
                for d in modes:
                    gs = {"one": self.graphs[(b, d)], **{n: alt[(b, d, n)] for n in variants[b]}}
                    for g in gs.values():  # warm every graph
                        g.replay()
                    torch.cuda.synchronize()
                    res = {n: [] for n in gs}
                    for _ in range(2):  # interleaved rounds, best of each
                        for n, g in gs.items():
                            res[n].append(timed(g))
                    times[(b, d)] = {n: min(v) for n, v in res.items()}

        # Each stage is agreed across ranks. prealloc (every allocation of the variants: their eager forwards with the
        # collectives skipped) and capture (records collectives, runs none) can fail on one rank without leaving
        # anything queued on its peers: every rank then keeps the all-reduce graphs. warm and measure RUN
        # collectives: if they fail on some rank after issuing part of them, its peers may hold collectives the failed
        # rank never joins (the native communicator has no device-side timeout), so every rank aborts the
        # communicator and raises instead of decoding on.
        def run_stages(pairs, triples, with_measure):
            stages = [("prealloc", lambda: forwards(pairs, True)), ("warm", lambda: forwards(pairs, False)),
                      ("capture", lambda: capture_all(triples))] + ([("measure", measure)] if with_measure else [])
            for name, stage in stages:
                ok, err = self.tp.agree(stage)
                if ok:
                    continue
                alt.clear()
                if name in ("prealloc", "capture"):
                    log.warning("decode schedule A/B stopped at %s (%s): every rank keeps the all-reduce schedule",
                                name, err or "on a peer rank")
                    buf.ctx.zero_()
                    buf.bt.zero_()
                    torch.cuda.synchronize()
                    return False
                self.tp.close(abort=True)
                raise RuntimeError(f"decode schedule A/B failed in {name} ({err or 'on a peer rank'}) after "
                                   f"collectives were issued: communicator aborted on every rank")
            return True

        pairs = [(b, n) for b in sorted(timed_b, reverse=True) for n in variants[b]]
        if not run_stages(pairs, [(b, d, n) for b, n in pairs for d in modes], True):
            return
        allt = self.tp.all_gather_object(times)
        win = {}
        for (b, d), tv in times.items():
            worst = {n: max(t[(b, d)][n] for t in allt) for n in tv}
            win[(b, d)] = min(worst, key=lambda n: worst[n] if n == "one" else worst[n] / 0.97)
            self.stats.setdefault("schedule_ab_ms", {})[f"{b}{'c' if d else 'g'}"] = \
                {n: round(v, 3) for n, v in worst.items()}
        # every candidate bucket: its own winner, or the nearest timed bucket's (when that schedule applies to it)
        chosen = {}
        for b in variants:
            near = min(timed_b, key=lambda t: (abs(t - b), t))
            for d in modes:
                w = win[(near, d)]
                if w != "one" and w in variants[b]:
                    chosen[(b, d)] = w
        extra = sorted({(b, d, n) for (b, d), n in chosen.items() if (b, d, n) not in alt}, reverse=True)
        for k in list(alt):  # timed alternatives that lost: free their graphs
            if chosen.get(k[:2]) != k[2]:
                del alt[k]
        if extra and not run_stages(sorted({(b, n) for b, _, n in extra}, reverse=True), extra, False):
            return
        for (b, d), best in chosen.items():
            self.graphs[(b, d)] = alt[(b, d, best)]
            if best == "rsag":  # eager steps of this bucket (none while its graph exists) take it too
                m.rsag.add(b)
            if best == "col":
                m.col.add(b)
            if self.decode_schedule.get(b, "one") == "one":
                self.decode_schedule[b] = best
        buf.ctx.zero_()
        buf.bt.zero_()
        torch.cuda.synchronize()
        log.info("decode schedule A/B (timed buckets %s, max over ranks, ms per step): %s -> %s", timed_b,
                 self.stats.get("schedule_ab_ms"), self.decode_schedule)

    # -------------------------------------------------------------------------- offline API
    def generate(self, prompts: Iterable[Sequence[int]], params=None) -> List[List[int]]:
        """Run a batch of prompts to completion; returns generated ids per prompt (in order)."""
        plist = list(prompts)
        if not isinstance(params, (list, tuple)):
            params = [params] * len(plist)
        rids = [self.add_request(p, sp) for p, sp in zip(plist, params)]
        while self.has_unfinished():
            self.step()
        out = [self.requests[r].output_ids for r in rids]
        for r in rids:
            self.requests.pop(r, None)
        return out
