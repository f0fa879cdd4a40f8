"""Data-parallel replicas behind one front-end (SURVEY 2.4 "DP replicas", optional).

Reference: none - its consumer notes that several subscribers *could* pop the same ``pqueue``
(consumer_server.py:68-72), but replies go to one shared, uncorrelated ``squeue``
(producer_server.py:50-53), so two consumers would swap answers.

Two forms, both with request-id correlation:

* across processes (``torchrun`` world = dp x tp, ``--dp``): every replica's leader runs a
  :class:`~llmss_amd.serving.consumer.Consumer` on the same broker; ``BRPOP pqueue`` is the load
  balancer (an idle replica pulls the next request) and each reply goes to ``squeue:<id>``;
* in one process (several single-GPU replicas, e.g. GPT-2-XL on every GPU of a node):
  :class:`Router` owns one :class:`EngineDriver` per replica and sends each request to the replica
  with the fewest requests in flight. It has the driver API the gRPC / HTTP front-ends use.
"""
from __future__ import annotations

import itertools
import threading
from typing import Callable, List, Optional

from ..engine.sampling import SamplingParams
from .driver import EngineDriver, Handle


class _Stats:
    def __init__(self, drivers):
        self._drivers = drivers

    @property
    def stats(self):
        out = {}
        for d in self._drivers:
            for k, v in d.engine.stats.items():
                if isinstance(v, (int, float)):
                    out[k] = out.get(k, 0) + v
        out["replicas"] = len(self._drivers)
        out["per_replica_tokens"] = [d.engine.stats.get("tokens", 0) for d in self._drivers]
        return out


class Router:
    leader = True

    def __init__(self, drivers: List[EngineDriver]):
        if not drivers:
            raise ValueError("Router needs at least one replica")
        self.drivers = drivers
        n = len(drivers)
        for i, d in enumerate(drivers):
            d.set_rid_space(i, n)  # request id -> replica = id % n
        self._rr = itertools.count()
        self._lock = threading.Lock()
        self.engine = _Stats(drivers)
        self.tp = drivers[0].tp
        self.routed = [0] * n

    @property
    def error(self):
        return next((d.error for d in self.drivers if d.error is not None), None)

    def _load(self, d: EngineDriver) -> int:
        return len(d.handles)

    def submit(self, prompt_ids, params: SamplingParams, on_done: Optional[Callable[[Handle], None]] = None,
               deadline_s: Optional[float] = None) -> Handle:
        with self._lock:
            live = [i for i, d in enumerate(self.drivers) if d.error is None] or list(range(len(self.drivers)))
            lo = min(self._load(self.drivers[i]) for i in live)
            least = [i for i in live if self._load(self.drivers[i]) == lo]
            i = least[next(self._rr) % len(least)]
            self.routed[i] += 1
            # submit under the lock: the chosen replica's load includes this request before the next pick
            return self.drivers[i].submit(prompt_ids, params, on_done=on_done, deadline_s=deadline_s)

    def abort(self, rid: int):
        self.drivers[rid % len(self.drivers)].abort(rid)

    def start(self):
        for d in self.drivers:
            d.start()
        return self

    def stop(self):
        for d in self.drivers:
            d.stop()

    def run(self):
        """Serve until stopped (the replicas' driver threads do the work)."""
        self.start()
        for d in self.drivers:
            d._thread.join()

    def generate(self, prompt_ids, params: SamplingParams, timeout: Optional[float] = None) -> Handle:
        h = self.submit(prompt_ids, params)
        if not h.wait(timeout):
            self.abort(h.rid)
            raise TimeoutError(f"request {h.rid} timed out")
        return h
