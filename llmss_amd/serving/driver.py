"""Tensor-parallel serving driver: the engine step loop on every rank + a CPU control plane.

Reference: the consumer broadcasts a pickled payload with ``dist.broadcast_object_list`` over the
NCCL world group on EVERY idle poll iteration (a spinning GPU collective, consumer_server.py:75-111,
quirk Q11), then runs one request at a time and broadcasts each sampled token (``:165``).

Here the leader (rank 0) owns admission; per engine step it sends the followers only the *new*
requests / aborts over a dedicated gloo (CPU/TCP) group, and all ranks then run an identical
``engine.step()`` (same scheduler decisions, same all-gathered logits, same Philox keys => same
tokens, no token broadcast). When there is no work the leader blocks on its inbox and followers
block in a CPU receive - nothing spins on the GPU.

Failure handling (the reference has none beyond the 60 s NCCL timeout):
* leader heartbeat: an idle leader still broadcasts a heartbeat every ``heartbeat_s``; followers
  wait on the control group with ``leader_timeout_s``, so a lost leader ends them cleanly instead
  of hanging in a collective forever.
* any exception in a step or a collective (a dead peer, a RCCL/gloo timeout) fails every
  in-flight request with ``finish_reason="error"`` and stops the driver on that rank.
* per-request deadlines (``submit(..., deadline_s=)``, gRPC deadlines) abort on every rank.
* fault injection for tests: ``LLMSS_FAULT_INJECT="rank:step:kind"`` (kind = exit | raise | hang)
  makes one rank misbehave at a given engine step.

Control channel: when every rank of the replica is on one host (always, for xGMI tensor parallelism)
the per-step record goes through a native shared-memory ring (csrc/ctrl.cpp ``CtrlRing``: the leader
writes, each follower reads at its own pace, ~microseconds per record) instead of a gloo TCP broadcast
(~0.1-0.3 ms per step at 2-8 ranks, profiles/r3_ctrl). ``LLMSS_CTRL=gloo`` forces the broadcast path;
ranks on several hosts fall back to it automatically.
"""
from __future__ import annotations

import collections
import gc
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from datetime import timedelta
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..engine.engine import LLMEngine
from ..engine.sampling import SamplingParams
from ..utils.logging import get_logger

log = get_logger(__name__)


@dataclass
class Handle:
    rid: int
    prompt_ids: List[int]
    params: SamplingParams
    tokens: "queue.Queue[Optional[int]]" = field(default_factory=queue.Queue)
    done: threading.Event = field(default_factory=threading.Event)
    output_ids: List[int] = field(default_factory=list)
    finish_reason: str = ""
    metrics: Dict[str, float] = field(default_factory=dict)
    on_done: Optional[Callable[["Handle"], None]] = None
    # streaming consumers only: tokens are queued for stream() (gRPC GenerateStream) and/or handed to
    # on_token; a unary request just accumulates output_ids (no per-token queue hop)
    stream: bool = False
    on_token: Optional[Callable[["Handle", int], None]] = None
    # batched delivery (gRPC streams): the step's tokens of every handle sharing a sink go to ONE
    # sink([(sink_q, token), ...]) call after the step, the finish marker as (sink_q, None) in order after
    # the handle's last token - one cross-thread wake-up per step instead of one per request
    sink: Optional[Callable[[list], None]] = None
    sink_q: object = None
    t_submit: float = field(default_factory=time.perf_counter)
    deadline: Optional[float] = None  # perf_counter time after which the request is aborted
    error: str = ""

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self.done.wait(timeout)

    def iter_tokens(self):
        """Tokens as they are sampled (submit(..., stream=True)); ends when the request finishes."""
        if not self.stream:
            raise RuntimeError("iter_tokens() needs a handle submitted with stream=True")
        while True:
            t = self.tokens.get()
            if t is None:
                return
            yield t


@dataclass
class FaultSpec:
    rank: int
    step: int
    kind: str  # exit | raise | hang

    @staticmethod
    def from_env() -> Optional["FaultSpec"]:
        v = os.environ.get("LLMSS_FAULT_INJECT")
        if not v:
            return None
        r, st, kind = v.split(":")
        return FaultSpec(int(r), int(st), kind)


class EngineDriver:
    def __init__(self, engine: LLMEngine, control_group=None, heartbeat_s: float = 1.0,
                 leader_timeout_s: float = 300.0, fault: Optional[FaultSpec] = None):
        self.engine = engine
        self.tp = engine.tp
        self.rank = self.tp.rank
        self.leader = self.rank == 0
        self.heartbeat_s = heartbeat_s
        self.cg = control_group
        if self.tp.is_real and self.cg is None:
            self.cg = getattr(self.tp, "ctrl_group", None) or \
                dist.new_group(backend="gloo", timeout=timedelta(seconds=leader_timeout_s))
        self.inbox: "queue.Queue" = queue.Queue()
        self.handles: Dict[int, Handle] = {}
        self._pending: Optional[dict] = None  # sink -> [(sink_q, token | None)] while a step's events are handed out
        self._next = 0
        self._stop = False
        self._thread: Optional[threading.Thread] = None
        self._lock = threading.Lock()
        self.idle_wait_s = 0.05
        # admission window: an idle leader that wakes on a request keeps collecting arrivals until none
        # came for `batch_window_s` (at most 10 windows) or the arrivals fill the free sequence slots, so a
        # burst of concurrent clients is admitted in one prefill step instead of trickling in one by one
        self.batch_window_s = float(os.environ.get("LLMSS_ADMIT_WINDOW_S", "0.003"))
        self.batch_window_max = 10
        # closed-loop clients send their next request as soon as a reply lands, but through the pub/sub path
        # (front-end -> broker -> consumer, two extra processes) a cohort's re-submissions reach the inbox spread
        # over more than one quiet period and used to split into cohorts that never re-align (profiles/r5_pubsub).
        # Two bounded corrections, both inside the batch_window_max * batch_window_s cap:
        # * `_expect` counts the replies of the last `resubmit_horizon_s` not yet matched by an arrival; while a
        #   window holds fewer arrivals than that, it tolerates a 4x longer gap between them and stays open up to
        #   `resubmit_windows` windows instead of batch_window_max (GPT-2-XL over pub/sub: 64 re-submissions
        #   arrive over 40-50 ms, profiles/r6_pubsub)
        # * near-drain hold: arrivals while every running sequence is within `merge_steps` tokens of its length
        #   limit wait (at most batch_window_max windows) for the engine to drain, so they prefill with the
        #   re-submissions of the sequences about to finish instead of one step ahead of them.
        self.resubmit_horizon_s = 0.25
        self.resubmit_windows = 25
        self.merge_steps = 2
        self._expect = 0
        self._expect_t = 0.0
        self._held: list = []  # inbox items held back by the near-drain rule, oldest first
        self._held_t = 0.0
        # the last admissions: (requests, engine was idle, window seconds, expected re-submissions) - diagnostics
        self.admit_log: "collections.deque" = collections.deque(maxlen=128)
        self.fault = fault if fault is not None else FaultSpec.from_env()
        self.error: Optional[BaseException] = None
        self._last_bcast = time.perf_counter()
        self.stats = {"ctrl_bcasts": 0, "ctrl_payloads": 0, "admit_windows": 0, "admit_window_s": 0.0,
                      "admit_window_reqs": 0, "admit_held": 0}
        self._rid_stride = 1
        # global rank of this replica's leader (broadcast src is a global rank in torch.distributed)
        self._src = dist.get_global_rank(self.cg, 0) if self.tp.is_real else 0
        self.leader_timeout_s = leader_timeout_s
        self._ring = self._open_ring() if self.tp.is_real else None
        self.ctrl = "shm-ring" if self._ring is not None else ("gloo" if self.tp.is_real else "local")

    def _open_ring(self):
        """Shared-memory control ring when every rank of the replica is on this host; None -> gloo.
        Collective over the control group: every rank reaches the same decision."""
        import socket
        import uuid

        if os.environ.get("LLMSS_CTRL", "shm").lower() == "gloo" or self.tp.size < 2:
            return None
        hosts = [None] * self.tp.size
        dist.all_gather_object(hosts, socket.gethostname(), group=self.cg)
        if len(set(hosts)) != 1:
            return None
        from .. import _native

        C = _native()
        ring, box = None, [""]
        if self.leader:
            name = f"/llmss_ctrl_{os.getpid()}_{uuid.uuid4().hex[:12]}"
            try:
                ring = C.CtrlRing(name, True, 1 << 24, self.tp.size - 1, 0)
                box[0] = name
            except Exception as e:  # noqa: BLE001 - no usable /dev/shm: everyone stays on gloo
                log.warning("control ring unavailable (%s); using gloo broadcasts", e)
        dist.broadcast_object_list(box, src=self._src, group=self.cg)
        ok = bool(box[0])
        if ok and not self.leader:
            try:
                ring = C.CtrlRing(box[0], False, 0, 0, self.rank - 1)
            except Exception as e:  # noqa: BLE001
                log.warning("rank %d: cannot attach control ring (%s)", self.rank, e)
                ok = False
        oks = [None] * self.tp.size
        dist.all_gather_object(oks, ok, group=self.cg)
        if not all(oks):
            return None  # the ring (if any) unmaps and unlinks when dropped
        if self.leader and not ring.wait_attached(60.0):
            raise RuntimeError("control ring: followers did not attach")
        return ring

    def set_rid_space(self, start: int, stride: int):
        """Request ids start, start + stride, ... (a Router keeps ids unique across its replicas)."""
        self._next, self._rid_stride = start, stride

    # --------------------------------------------------------------------- leader API
    def submit(self, prompt_ids: List[int], params: SamplingParams,
               on_done: Optional[Callable[[Handle], None]] = None, deadline_s: Optional[float] = None,
               stream: bool = False, on_token: Optional[Callable[[Handle, int], None]] = None,
               sink: Optional[Callable[[list], None]] = None, sink_q=None) -> Handle:
        if not self.leader:
            raise RuntimeError("submit() is only valid on rank 0")
        params.resolved_seed()  # fix the seed on the leader so every rank uses the same one
        with self._lock:
            rid = self._next
            self._next += self._rid_stride
        h = Handle(rid, list(prompt_ids), params, on_done=on_done, stream=stream, on_token=on_token, sink=sink,
                   sink_q=sink_q)
        if deadline_s is not None:
            h.deadline = h.t_submit + deadline_s
        if self.error is not None:  # the driver already failed: refuse instead of queueing forever
            h.error = f"driver stopped: {self.error}"
            self._complete(h, "error")
            return h
        self.handles[rid] = h
        self.inbox.put(("new", h))
        return h

    def abort(self, rid: int):
        self.inbox.put(("abort", rid))

    def stop(self):
        self._stop = True
        self.inbox.put(("stop", None))
        if self._thread is not None:
            self._thread.join(timeout=60)

    def start(self):
        self._thread = threading.Thread(target=self.run, daemon=True, name=f"engine-driver-r{self.rank}")
        self._thread.start()
        return self

    # --------------------------------------------------------------------- loop
    _EMPTY = {"new": [], "abort": [], "stop": False}

    def _bcast(self, msg):
        """Leader -> followers, once per engine step. The common case (nothing new) costs one 16-byte
        gloo broadcast of a fixed-size header; the pickled payload follows only when the step
        admits or aborts requests (the reference pickles a broadcast_object_list on every idle poll,
        consumer_server.py:108)."""
        if not self.tp.is_real:
            return msg
        import pickle

        if self._ring is not None:  # one record per step: 1 byte when nothing is new
            self.stats["ctrl_bcasts"] += 1
            if self.leader:
                if not msg["new"] and not msg["abort"] and not msg["stop"]:
                    self._ring.send(b"\x01" if msg.get("hb") else b"\x00", self.leader_timeout_s)
                else:
                    self.stats["ctrl_payloads"] += 1
                    self._ring.send(b"\x02" + pickle.dumps(msg, protocol=pickle.HIGHEST_PROTOCOL),
                                    self.leader_timeout_s)
                return msg
            rec = self._ring.recv(self.leader_timeout_s)
            if rec[:1] != b"\x02":
                return dict(self._EMPTY, hb=rec[:1] == b"\x01")
            self.stats["ctrl_payloads"] += 1
            return pickle.loads(rec[1:])
        hdr = torch.zeros(2, dtype=torch.int64)
        payload = None
        if self.leader:
            empty = not msg["new"] and not msg["abort"] and not msg["stop"]
            if not empty:
                payload = pickle.dumps(msg, protocol=pickle.HIGHEST_PROTOCOL)
                hdr[0] = len(payload)
            hdr[1] = 1 if msg.get("hb") else 0
        dist.broadcast(hdr, src=self._src, group=self.cg)
        n = int(hdr[0])
        self.stats["ctrl_bcasts"] += 1
        if n == 0:
            return dict(self._EMPTY, hb=bool(hdr[1]))
        self.stats["ctrl_payloads"] += 1
        buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if self.leader else torch.empty(n, dtype=torch.uint8)
        dist.broadcast(buf, src=self._src, group=self.cg)
        return msg if self.leader else pickle.loads(buf.numpy().tobytes())

    def _next_item(self, timeout: Optional[float]):
        """The oldest held-back item, else the inbox's (waiting up to `timeout`; None = do not wait)."""
        if self._held:
            return self._held.pop(0)
        return self.inbox.get_nowait() if timeout is None else self.inbox.get(timeout=timeout)

    def _near_drain(self) -> bool:
        """Nothing waits and every running sequence is within merge_steps tokens of its length limit."""
        sch = self.engine.sched
        if sch.num_waiting() or not sch.num_running():
            return False
        lim = self.merge_steps
        return all(r.finished or len(r.output_ids) + lim >= r.params.max_new_tokens
                   for r in self.engine.requests.values())

    def _collect(self, block: bool):
        """Leader: drain the held-back items and the inbox (blocking when idle). Returns a control message."""
        new, raw, aborts, stop = [], [], [], False
        held = bool(self._held)
        now = time.perf_counter()
        expect = self._expect if now - self._expect_t < self.resubmit_horizon_s else 0
        t_start = self._held_t if held else now
        try:
            item = self._next_item(self.idle_wait_s if block and not held else None)
            if not held:
                t_start = time.perf_counter()
            t_end = t_start + self.batch_window_max * self.batch_window_s
            # a burst that fills every free sequence slot closes the window at once: a later arrival could not
            # join this prefill step anyway
            sch = self.engine.sched
            cap = self.engine.max_num_seqs - sch.num_waiting() - sch.num_running()
            while True:
                kind, v = item
                if kind == "new":
                    new.append((v.rid, v.prompt_ids, v.params.__dict__.copy()))
                    raw.append(item)
                elif kind == "abort":
                    aborts.append(v)
                elif kind == "stop":
                    stop = True
                try:
                    item = self._next_item(None)
                except queue.Empty:
                    short = len(new) < expect  # replies whose re-submission has not arrived yet
                    lim = t_start + self.resubmit_windows * self.batch_window_s if short else t_end
                    if not (block and self.batch_window_s > 0 and new and not stop) or time.perf_counter() > lim \
                            or len(new) >= cap:
                        raise
                    item = self.inbox.get(timeout=self.batch_window_s * (4 if short else 1))
        except queue.Empty:
            pass
        if new and not block and not stop and time.perf_counter() < t_end and self._near_drain():
            # hold the arrivals back until the engine drains (or the cap): they join the next idle window
            gone = set(aborts)
            self._held = [it for it in raw if it[1].rid not in gone]
            self._held_t = t_start
            self.stats["admit_held"] += 0 if held else 1
            new = []
        elif new:
            self._expect = max(0, expect - len(new))
            self.admit_log.append((len(new), block, round(time.perf_counter() - t_start, 4), expect))
        if block and new:
            self.stats["admit_windows"] += 1
            self.stats["admit_window_s"] += time.perf_counter() - t_start
            self.stats["admit_window_reqs"] += len(new)
        now = time.perf_counter()
        for h in list(self.handles.values()):  # server-side deadlines
            if h.deadline is not None and now > h.deadline and h.rid not in aborts:
                h.error = "deadline exceeded"
                aborts.append(h.rid)
        return {"new": new, "abort": aborts, "stop": stop}

    def _inject(self, step: int):
        f = self.fault
        if f is None or f.rank != self.rank or step != f.step:
            return
        log.warning("rank %d: injecting fault %r at step %d", self.rank, f.kind, step)
        if f.kind == "exit":
            os._exit(17)
        if f.kind == "hang":
            while True:
                time.sleep(3600)
        raise RuntimeError(f"injected fault at step {step}")

    def run(self):
        if self.engine.is_gpu:
            # a serving process keeps its model, KV pool, plans and graphs for its lifetime: move them out of
            # the cyclic collector's generations so a full collection while serving scans only per-request
            # objects (served GPT-2-XL steps showed ~110-130 ms stalls on 2 of 20 steps)
            gc.collect()
            gc.freeze()
        try:
            self._run()
        except Exception as e:  # noqa: BLE001 - a dead peer, a collective timeout, a kernel error
            self.error = e
            log.error("rank %d: engine driver stopped: %s", self.rank, e)
            for h in list(self.handles.values()):
                h.error = h.error or f"engine failure: {e}"
                self._complete(h, "error")
        finally:
            if self._ring is not None and self.leader:
                self._ring.close_producer()  # followers still waiting see "producer closed" at once

    def _run(self):
        eng = self.engine
        dev_ok = eng.is_gpu
        if dev_ok:
            torch.cuda.set_device(eng.device)
        steps = 0
        while True:
            if self.leader:
                # idle = no sequence left to schedule. A speculatively launched decode step may still be in flight
                # (pipelined decode; its rows all finished): it is collected on the next step, and a request
                # burst arriving meanwhile still gets the admission window, i.e. lands in one prefill step
                idle = not eng.sched.has_work()
                msg = self._collect(block=idle)
                if msg["new"]:
                    self.stats["admit_steps"] = self.stats.get("admit_steps", 0) + 1
                quiet = not msg["new"] and not msg["abort"] and not msg["stop"] and not self._stop
                if idle and quiet and not eng.has_unfinished():
                    if not self.tp.is_real or time.perf_counter() - self._last_bcast < self.heartbeat_s:
                        continue  # nothing to do, nothing to tell the followers
                    msg["hb"] = True  # heartbeat: followers time out if the leader disappears
            else:
                msg = None
            msg = self._bcast(msg)
            self._last_bcast = time.perf_counter()
            for rid, prompt, pd in msg["new"]:
                try:
                    eng.add_request(prompt, SamplingParams(**pd), req_id=rid)
                except ValueError as e:
                    # the validation is deterministic, so every rank rejects the same request: it fails on its
                    # own handle and the replica keeps serving the rest
                    log.warning("rank %d: request %d rejected: %s", self.rank, rid, e)
                    h = self.handles.get(rid) if self.leader else None
                    if h is not None:
                        h.error = f"rejected: {e}"
                        self._complete(h, "error")
            for rid in msg["abort"]:
                eng.abort(rid)
                self._finish_abort(rid)
            if msg["stop"]:
                break
            if not eng.has_unfinished():
                continue
            self._inject(steps)
            events = eng.step()
            steps += 1
            if self.leader:
                self._pending = {}
                try:
                    for ev in events:
                        h = self.handles.get(ev.req_id)
                        if h is None:
                            continue
                        h.output_ids.append(ev.token)
                        if h.stream:
                            h.tokens.put(ev.token)
                        if h.on_token is not None:
                            h.on_token(h, ev.token)
                        if h.sink is not None:
                            self._pending.setdefault(h.sink, []).append((h.sink_q, ev.token))
                        if ev.finished:
                            self._complete(h, ev.finish_reason)
                finally:
                    pending, self._pending = self._pending, None
                    for sink, items in pending.items():
                        sink(items)
            for r in eng.pop_finished():
                pass

    def _complete(self, h: Handle, reason: str):
        req = self.engine.requests.get(h.rid)
        h.finish_reason = reason
        if req is not None:
            h.metrics = req.metrics()
        if reason not in ("error", "abort", "deadline"):  # a closed-loop client's next request is on its way
            now = time.perf_counter()
            self._expect = (self._expect if now - self._expect_t < self.resubmit_horizon_s else 0) + 1
            self._expect_t = now
        if h.stream:
            h.tokens.put(None)
        if h.sink is not None:
            if self._pending is not None:  # inside a step: after this handle's last token
                self._pending.setdefault(h.sink, []).append((h.sink_q, None))
            else:
                h.sink([(h.sink_q, None)])
        h.done.set()
        self.handles.pop(h.rid, None)
        if h.on_done is not None:
            try:
                h.on_done(h)
            except Exception:  # noqa: BLE001
                log.exception("on_done callback failed")

    def _finish_abort(self, rid):
        h = self.handles.get(rid)
        if h is not None:
            self._complete(h, "deadline" if h.error == "deadline exceeded" else "abort")

    # --------------------------------------------------------------------- convenience
    def generate(self, prompt_ids: List[int], params: SamplingParams, timeout: Optional[float] = None) -> Handle:
        h = self.submit(prompt_ids, params)
        if not h.wait(timeout):
            self.abort(h.rid)
            raise TimeoutError(f"request {h.rid} timed out")
        return h
