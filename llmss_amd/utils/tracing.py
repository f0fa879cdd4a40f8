"""Tracing / profiling hooks (reference has none beyond a rank-0 wall clock, generate.py:44-45).

* :func:`range` - roctx push/pop ranges (``librocprofiler-sdk-roctx`` via ctypes) so engine phases
  (prefill, decode, sample, all-reduce) show up in ``rocprofv3 --marker-trace`` timelines.
  Enabled with ``LLMSS_ROCTX=1``; a no-op otherwise (no per-step cost).
* :class:`PhaseTimer` - HIP-event timers accumulated per phase (device time, no host sync until
  :meth:`summary`), enabled with ``LLMSS_TIMING=1``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from collections import defaultdict
from typing import Dict, List, Tuple

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("LLMSS_ROCTX") == "1":
            for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _ROCTX = lib
                    break
                except OSError:
                    continue
    return _ROCTX


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors roctx naming)
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class PhaseTimer:
    def __init__(self, enabled: bool = None):
        self.enabled = (os.environ.get("LLMSS_TIMING") == "1") if enabled is None else enabled
        self.pending: List[Tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled or not torch.cuda.is_available():
            with range(name):
                yield
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        with range(name):
            yield
        e.record()
        self.pending.append((name, s, e))

    def summary(self) -> Dict[str, Dict[str, float]]:
        if self.pending:
            torch.cuda.synchronize()
            for name, s, e in self.pending:
                self.totals[name] += s.elapsed_time(e)
                self.counts[name] += 1
            self.pending.clear()
        return {k: {"total_ms": round(v, 3), "count": self.counts[k], "avg_ms": round(v / self.counts[k], 4)}
                for k, v in self.totals.items()}
