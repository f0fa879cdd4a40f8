"""Continuous-batching generation engine (one instance per tensor-parallel rank).

Reference counterpart: the decode loops inlined in ``generate.py:99-190`` and
``consumer_server.py:114-166`` - one batch at a time, KV cache grown with ``torch.cat``,
sampling on rank 0 followed by a ``dist.broadcast`` of the token every step, a host sync per
token and (no-cache mode) ``torch.cuda.empty_cache()`` per token.

Here:
* the C++ :class:`Scheduler` admits prompts FCFS under token/sequence/KV-block budgets and
  batches every running sequence's next token (continuous batching, preemption by recompute);
* the KV cache is a preallocated paged pool sized from free HBM (288 GB per MI355X);
* decode steps replay a HIP graph captured per batch-size bucket (embedding -> all layers incl.
  RCCL all-reduces -> LM head -> all-gather -> sampler), so a step is one graph launch;
* every rank runs the same scheduler on the same request stream and samples the same token
  from the same all-gathered logits with the same per-step Philox key - no token broadcast.
"""
from __future__ import annotations

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
from .sampling import SamplingParams, step_seed

log = get_logger(__name__)


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
    """Static device buffers (+ pinned host mirrors) feeding the captured decode graphs."""

    def __init__(self, max_b: int, max_blocks: int, device):
        self.max_b, self.max_blocks = max_b, max_blocks
        pin = torch.cuda.is_available() and device.type == "cuda"
        self.h_i64 = torch.zeros(4 * max_b, dtype=torch.int64, pin_memory=pin)  # ids|pos|slots|seeds
        self.h_i32 = torch.zeros(2 * max_b + max_b * max_blocks, dtype=torch.int32, pin_memory=pin)  # ctx|topk|bt
        self.h_f32 = torch.zeros(2 * max_b, dtype=torch.float32, pin_memory=pin)  # temp|topp
        self.d_i64 = torch.zeros_like(self.h_i64, device=device)
        self.d_i32 = torch.zeros_like(self.h_i32, device=device)
        self.d_f32 = torch.zeros_like(self.h_f32, device=device)
        self.out = torch.zeros(max_b, dtype=torch.int64, device=device)
        self.h_out = torch.zeros(max_b, dtype=torch.int64, pin_memory=pin)
        B = max_b
        self.ids, self.pos, self.slots, self.seeds = (self.d_i64[i * B:(i + 1) * B] for i in range(4))
        self.ctx, self.topk = self.d_i32[:B], self.d_i32[B:2 * B]
        self.bt = self.d_i32[2 * B:].view(B, max_blocks)
        self.temp, self.topp = self.d_f32[:B], self.d_f32[B:]

    def fill(self, b_pad, ids, pos, slots, seeds, ctx, topk, bt, temp, topp):
        n = len(ids)
        B, MB = self.max_b, self.max_blocks
        hi = self.h_i64.numpy()
        hi32 = self.h_i32.numpy()
        hf = self.h_f32.numpy()
        for j, arr in enumerate((ids, pos, slots, seeds)):
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
        self.d_i64.copy_(self.h_i64, non_blocking=True)
        self.d_i32.copy_(self.h_i32, non_blocking=True)
        self.d_f32.copy_(self.h_f32, non_blocking=True)


class LLMEngine:
    def __init__(self, model: DecoderLM, *, max_num_seqs: int = 256, max_batched_tokens: int = 8192,
                 block_size: int = 16, num_blocks: Optional[int] = None, max_model_len: Optional[int] = None,
                 kv_fraction: float = 0.9, use_graphs: Optional[bool] = None, eos_token_id: Optional[int] = None,
                 graph_buckets: Optional[Sequence[int]] = None, check_tokens: Optional[bool] = None,
                 autotune: Optional[bool] = None):
        self.model = model
        self.cfg = model.cfg
        self.tp = model.tp
        self.device = model.device
        self.is_gpu = self.device.type == "cuda"
        self.block_size = block_size
        self.max_model_len = min(max_model_len or self.cfg.max_position_embeddings, self.cfg.max_position_embeddings)
        self.max_num_seqs = max_num_seqs
        self.max_batched_tokens = max(max_batched_tokens, self.max_model_len)
        self.eos = eos_token_id if eos_token_id is not None else self.cfg.eos_token_id
        self.max_blocks = math.ceil(self.max_model_len / block_size)
        self.num_blocks = num_blocks or self._auto_blocks(kv_fraction)
        self.kv = model.allocate_kv_cache(self.num_blocks, block_size)
        self.sched = _native().Scheduler(self.num_blocks, block_size, max_num_seqs, self.max_batched_tokens,
                                         self.max_model_len)
        self.requests: Dict[int, Request] = {}
        self._next_id = 0
        self.check_tokens = check_tokens if check_tokens is not None else os.environ.get("LLMSS_CHECK_TOKENS") == "1"
        self.stats = {"steps": 0, "prefill_steps": 0, "decode_steps": 0, "tokens": 0, "prefill_tokens": 0,
                      "preemptions": 0, "decode_time_s": 0.0, "prefill_time_s": 0.0}
        self.timer = PhaseTimer()  # LLMSS_TIMING=1: HIP-event device time per phase; LLMSS_ROCTX=1: roctx ranges
        self.use_graphs = self.is_gpu if use_graphs is None else (use_graphs and self.is_gpu)
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.buckets = sorted(set(graph_buckets or self._default_buckets()))
        self.buckets = [b for b in self.buckets if b <= max_num_seqs] or [max_num_seqs]
        if self.buckets[-1] < max_num_seqs:
            self.buckets.append(max_num_seqs)
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
        if self.use_graphs and os.environ.get("LLMSS_GRAPHS", "1") == "0":
            self.use_graphs = False
        if self.use_graphs:
            try:
                self.capture_graphs()
            except RuntimeError as e:  # e.g. a collective backend that refuses stream capture
                log.warning("decode graph capture failed (%s): running decode eagerly", e)
                torch.cuda.synchronize()
                self.graphs.clear()
                self.use_graphs = False

    # -------------------------------------------------------------------------- sizing
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
        buckets that DecoderLM splits for all-reduce / compute overlap."""
        out = set(self.buckets)
        for b in self.buckets:
            h = self.model.overlap_split(b)
            if h:
                out.update((h, b - h))
        return sorted(out)

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
        self.requests[rid] = req
        self.sched.add(rid, len(prompt), max_new)
        return rid

    def abort(self, rid: int):
        if rid in self.requests:
            self.sched.abort(rid)
            r = self.requests[rid]
            r.finished, r.finish_reason = True, "abort"

    def has_unfinished(self) -> bool:
        return self.sched.has_work()

    def pop_finished(self) -> List[Request]:
        done = [r for r in self.requests.values() if r.finished]
        for r in done:
            del self.requests[r.id]
        return done

    # -------------------------------------------------------------------------- step
    def _sampling_arrays(self, reqs: List[Request]):
        temp = np.array([r.params.k_temperature for r in reqs], dtype=np.float32)
        topk = np.array([r.params.k_top_k for r in reqs], dtype=np.int32)
        topp = np.array([r.params.k_top_p for r in reqs], dtype=np.float32)
        seeds = np.array([step_seed(r.seed, len(r.output_ids)) for r in reqs], dtype=np.int64)
        return temp, topk, topp, seeds

    def step(self) -> List[StepEvent]:
        with trace_range("schedule"):
            batch = self.sched.schedule()
        if batch.kind == 0:
            return []
        for rid in batch.preempted.tolist():
            self.stats["preemptions"] += 1
        ids = batch.ids.tolist()
        reqs = [self.requests[i] for i in ids]
        t0 = time.perf_counter()
        if batch.kind == 1:
            with self.timer.phase("prefill"):
                tokens = self._prefill(batch, reqs)
            self.stats["prefill_steps"] += 1
            self.stats["prefill_tokens"] += int(batch.query_lens.sum())
        else:
            with self.timer.phase("decode"):
                tokens = self._decode(batch, reqs)
            self.stats["decode_steps"] += 1
        if self.check_tokens and self.tp.is_real:
            allt = self.tp.all_gather_object(tokens)
            if any(t != tokens for t in allt):
                raise RuntimeError(f"rank {self.tp.rank}: sampled tokens diverged across TP ranks: {allt}")
        now = time.perf_counter()
        self.stats["decode_time_s" if batch.kind == 2 else "prefill_time_s"] += now - t0
        self.stats["steps"] += 1
        events = []
        for r, tok in zip(reqs, tokens):
            r.output_ids.append(tok)
            if not r.t_first:
                r.t_first = now
            r.t_last = now
            r.token_times.append(now)
            self.stats["tokens"] += 1
            reason = ""
            if len(r.output_ids) >= r.params.max_new_tokens:
                reason = "length"
            elif not r.params.ignore_eos and self.eos is not None and tok == self.eos:
                reason = "eos"
            elif tok in r.params.stop_token_ids:
                reason = "stop"
            fin = bool(reason)
            self.sched.on_token(r.id, fin)
            if fin:
                r.finished, r.finish_reason = True, reason
            events.append(StepEvent(r.id, tok, fin, reason))
        return events

    def _prefill(self, batch, reqs: List[Request]) -> List[int]:
        dev = self.device
        qlens = batch.query_lens.astype(np.int64)
        ids = np.concatenate([np.asarray(r.all_ids[:q], dtype=np.int64) for r, q in zip(reqs, qlens)])
        cu = np.zeros(len(reqs) + 1, dtype=np.int32)
        cu[1:] = np.cumsum(qlens)
        inp = StepInput(
            kind="prefill",
            input_ids=torch.from_numpy(ids).to(dev, non_blocking=True),
            positions=torch.from_numpy(batch.positions).to(dev, non_blocking=True),
            slots=torch.from_numpy(batch.slots).to(dev, non_blocking=True),
            cu_seqlens=torch.from_numpy(cu).to(dev, non_blocking=True),
            max_seqlen=int(qlens.max()),
            last_idx=torch.from_numpy(cu[1:].astype(np.int64) - 1).to(dev, non_blocking=True),
        )
        logits = self.model(inp, self.kv)
        temp, topk, topp, seeds = self._sampling_arrays(reqs)
        tok = ops.sample(logits, torch.from_numpy(temp).to(dev), torch.from_numpy(topk).to(dev),
                         torch.from_numpy(topp).to(dev), torch.from_numpy(seeds).to(dev),
                         vocab=min(self.cfg.vocab_size, logits.shape[-1]))
        return tok.cpu().tolist()

    def _decode_forward(self, b: int, buf: _DecodeBuffers):
        inp = StepInput(kind="decode", input_ids=buf.ids[:b], positions=buf.pos[:b], slots=buf.slots[:b],
                        block_tables=buf.bt[:b], ctx_lens=buf.ctx[:b], max_ctx=self.max_model_len,
                        decode_splits=self._splits(b))
        logits = self.model(inp, self.kv)
        _hip_ops.sample(logits, buf.temp[:b], buf.topk[:b], buf.topp[:b], buf.seeds[:b],
                        vocab=min(self.cfg.vocab_size, logits.shape[-1]), out=buf.out[:b])

    def _decode(self, batch, reqs: List[Request]) -> List[int]:
        n = len(reqs)
        ids = np.array([r.last_id for r in reqs], dtype=np.int64)
        temp, topk, topp, seeds = self._sampling_arrays(reqs)
        if not self.is_gpu:
            dev = self.device
            inp = StepInput(kind="decode", input_ids=torch.from_numpy(ids), positions=torch.from_numpy(batch.positions),
                            slots=torch.from_numpy(batch.slots),
                            block_tables=torch.from_numpy(batch.block_table.astype(np.int32)),
                            ctx_lens=torch.from_numpy(batch.ctx_lens.astype(np.int32)), max_ctx=self.max_model_len)
            logits = self.model(inp, self.kv)
            return ops.sample(logits, temp, topk, topp, seeds, vocab=min(self.cfg.vocab_size, logits.shape[-1])).tolist()
        b = next(x for x in self.buckets if x >= n)
        self.buf.fill(b, ids, batch.positions, batch.slots, seeds, batch.ctx_lens, topk, batch.block_table, temp, topp)
        if self.use_graphs and b in self.graphs:
            self.graphs[b].replay()
        else:
            self._decode_forward(b, self.buf)
        self.buf.h_out[:n].copy_(self.buf.out[:n], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return self.buf.h_out[:n].tolist()

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
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for b in reversed(self.buckets):
                for _ in range(2):
                    self._decode_forward(b, buf)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for b in reversed(self.buckets):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                self._decode_forward(b, buf)
            self.graphs[b] = g
        torch.cuda.synchronize()
        log.info("captured %d decode graphs: %s", len(self.graphs), self.buckets)

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
