"""Process-group bootstrap and the tensor-parallel communicator.

Reference: ``src/llmss/server/models/utils/dist.py:40-77`` (``initialize_torch_distributed``)
and ``FakeGroup`` (``dist.py:14-37``). Differences, by design:

* One process per GPU; the device is chosen from ``LOCAL_RANK`` (not ``RANK % count``) so the
  same code runs on one node or several.
* ``world_size == 1`` is a first-class case: :class:`TPGroup` with ``size == 1`` turns every
  collective into the identity and *never* needs a default process group (the reference's
  single-GPU ``generate.py`` crashes on an un-grouped ``dist.broadcast`` — SURVEY Q2).
* On GPUs the data plane is a native RCCL communicator (``llmss_amd._C.RcclComm``, csrc/comm.cpp)
  bootstrapped over a CPU (gloo) process group: collectives are raw ``ncclAllReduce`` /
  ``ncclAllGather`` calls on the caller's current HIP stream, so they are captured into the decode
  HIP graphs with the rest of the step, with no torch Work / event / watchdog in the loop.
  ``LLMSS_COMM=torch`` selects torch's ``nccl`` process group instead (RCCL as well), created with
  the reference's high-priority-stream option (``dist.py:52-53``).
* ``DEBUG=1`` keeps the reference's "fake" semantics: every rank computes with its own shard and
  no communication happens (shape/loader debugging only, numerically wrong by construction).
"""
from __future__ import annotations

import contextlib
import os
from datetime import timedelta
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..utils.logging import get_logger

log = get_logger(__name__)


class TPGroup:
    """Tensor-parallel communicator (size 1, real, or fake)."""

    def __init__(self, rank: int = 0, size: int = 1, group=None, fake: bool = False,
                 sim_comm: Optional[Tuple[float, float]] = None, comm=None):
        self.rank = rank
        self.size = size
        self.group = group
        self.fake = fake
        # native RCCL communicator (device tensors); `group` then is the CPU (gloo) group of the same ranks
        self.comm = comm
        self._suspend = False  # suspended(): data-plane collectives are skipped (shape-only warm-up)
        # fake groups only: (latency us, algorithmic GB/s[, channels]) of a modelled all-reduce. Each all-reduce
        # then occupies the issuing stream for latency + bytes/bandwidth, so the comm/compute overlap of a TP=N
        # schedule can be measured on one GPU: a spin kernel on one workgroup, or with `channels` the many-CU model
        # (csrc/comm_model.hip: that many workgroups moving the collective's local memory traffic, as RCCL's do).
        self.sim_comm = sim_comm if fake and size > 1 else None
        # fake groups standing in for a TP=N rank (bench --simulate-tp): all-gathers return N copies of the
        # local shard, so what consumes them (the candidate sampler's N groups, a full-width logits row)
        # costs what it costs at TP=N. Off for DEBUG=1 (the reference FakeGroup returns the local tensor).
        self.replicate_gather = False
        self._cycles_per_us = None
        # data parallelism (initialize_distributed(dp=...)): this group is replica `replica` of `dp`
        self.replica, self.dp, self.global_rank, self.ctrl_group = 0, 1, rank, None

    # reference-compatible accessors (FakeGroup.size()/rank())
    def world_size(self) -> int:
        return self.size

    @property
    def is_real(self) -> bool:
        return self.size > 1 and not self.fake

    @property
    def comm_active(self) -> bool:
        """Collectives take time on a stream (real communicator, or a fake one modelling comm)."""
        return self.is_real or self.sim_comm is not None

    def _sim_wait(self, nbytes: int):
        if self._cycles_per_us is None:  # calibrate the spin kernel's clock once (outside capture)
            torch.cuda._sleep(1000)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            torch.cuda._sleep(2_000_000)
            e.record()
            e.synchronize()
            self._cycles_per_us = 2_000_000 / (s.elapsed_time(e) * 1e3)
        lat, gbps = self.sim_comm[:2]
        us = lat + nbytes / (gbps * 1e3)
        if len(self.sim_comm) > 2:
            from .. import _native

            lib, ch = _native(), int(self.sim_comm[2])
            buf = getattr(self, "_sim_buf", None)
            if buf is None:
                # sized once for the largest slice (comm_model_slice caps it), never re-allocated: graphs captured
                # earlier keep its address, so freeing it for a larger collective would leave them writing into
                # memory the allocator has handed out again
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("modelled-collective scratch must be allocated before graph capture")
                buf = self._sim_buf = torch.empty(ch * 2 * lib.comm_model_slice(ch, 1 << 40), dtype=torch.uint8,
                                                  device="cuda")
            if buf.numel() < ch * 2 * lib.comm_model_slice(ch, nbytes):
                raise RuntimeError("modelled-collective scratch too small")
            lib.comm_model(buf.data_ptr(), ch, nbytes, us, torch.cuda.current_stream().cuda_stream)
            return
        torch.cuda._sleep(max(1, int(us * self._cycles_per_us)))

    @property
    def host_staged(self) -> bool:
        """gloo group: device tensors go through host copies (gloo has no device all-gather).

        Only the multi-rank-on-one-GPU tests use this (several TP ranks sharing the development
        box's single MI355X); the RCCL data plane never stages.
        """
        st = getattr(self, "_host_staged", None)
        if st is None:
            st = self._host_staged = self.is_real and self.comm is None and dist.get_backend(self.group) == "gloo"
        return st

    @property
    def backend(self) -> str:
        """'rccl-native' | 'nccl' (torch's RCCL process group) | 'gloo' | 'local' | 'fake'."""
        if self.fake:
            return "fake"
        if not self.is_real:
            return "local"
        return "rccl-native" if self.comm is not None else dist.get_backend(self.group)

    def _native_ok(self, t: torch.Tensor) -> bool:
        return self.comm is not None and t.is_cuda

    @staticmethod
    def _code(t: torch.Tensor) -> int:
        from .. import _native

        return _native().rccl_dtypes[str(t.dtype).replace("torch.", "")]

    @staticmethod
    def _no_capture():
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("host-staged (gloo) collectives cannot be captured into a HIP graph; "
                               "run the engine with use_graphs=False on this group")

    @contextlib.contextmanager
    def suspended(self):
        """Skip the data-plane collectives inside the block (every rank must do the same): all_reduce
        returns its input, all_gather_last_dim N copies of the local shard. For warm-up passes whose
        values are discarded but whose collectives would otherwise leave work items in torch's RCCL
        watchdog right before a graph capture (torch process-group mode only)."""
        prev, self._suspend = self._suspend, True
        try:
            yield self
        finally:
            self._suspend = prev

    # ------------------------------------------------------------ data plane
    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self._suspend:
            return t
        if self.is_real and self._native_ok(t):
            if not t.is_contiguous():
                raise ValueError("all_reduce needs a contiguous tensor")
            self.comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._code(t),
                                 torch.cuda.current_stream().cuda_stream)
        elif self.is_real and t.is_cuda and self.host_staged:
            self._no_capture()
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        elif self.is_real:
            dist.all_reduce(t, group=self.group)
        elif self.sim_comm is not None and t.is_cuda:
            self._sim_wait(t.numel() * t.element_size())
        return t

    def all_gather_last_dim(self, t: torch.Tensor) -> torch.Tensor:
        """Gather shards along the last dim: [..., n] -> [..., size*n]."""
        if self._suspend and self.size > 1:
            return torch.cat([t.contiguous()] * self.size, -1)
        if not self.is_real:
            if self.sim_comm is not None and t.is_cuda:
                self._sim_wait(self.size * t.numel() * t.element_size())
            if self.replicate_gather and self.size > 1:
                return torch.cat([t] * self.size, -1)
            return t
        t = t.contiguous()
        if self._native_ok(t):
            out = torch.empty((self.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), self._code(t),
                                 torch.cuda.current_stream().cuda_stream)
        elif t.is_cuda and self.host_staged:
            self._no_capture()
            h = t.cpu()
            out = torch.empty((self.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype)
            dist.all_gather_into_tensor(out, h, group=self.group)
            out = out.to(t.device)
        else:
            out = torch.empty((self.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t, group=self.group)
        out = out.view((self.size,) + tuple(t.shape))
        return out.movedim(0, -2).reshape(*t.shape[:-1], self.size * t.shape[-1])

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Sum ``t`` ([M, ...], M % size == 0) over the ranks and return this rank's block of M / size rows
        (RCCL reduce-scatter; the row-sharded decode schedule of DecoderLM). Fake / suspended groups return
        the local block (a modelled group spends the collective's time first)."""
        n = self.size
        if t.shape[0] % n:
            raise ValueError(f"reduce_scatter_rows: {t.shape[0]} rows do not split over {n} ranks")
        m = t.shape[0] // n
        if self._suspend or not self.is_real:
            if self.sim_comm is not None and t.is_cuda and not self._suspend:
                self._sim_wait(t.numel() * t.element_size() // max(1, n))
            return t[self.rank * m:(self.rank + 1) * m]
        t = t.contiguous()
        out = torch.empty((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if self._native_ok(t):
            self.comm.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), self._code(t),
                                     torch.cuda.current_stream().cuda_stream)
        elif t.is_cuda and self.host_staged:
            self._no_capture()
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            out.copy_(h[self.rank * m:(self.rank + 1) * m])
        elif dist.get_backend(self.group) == "gloo":  # gloo has no reduce-scatter: all-reduce, keep the block
            h = t.clone()
            dist.all_reduce(h, group=self.group)
            out.copy_(h[self.rank * m:(self.rank + 1) * m])
        else:
            dist.reduce_scatter_tensor(out, t, group=self.group)
        return out

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """[m, ...] on every rank -> [size * m, ...], rank r's rows at block r (RCCL all-gather). Fake /
        suspended groups return ``size`` copies of the local block."""
        n = self.size
        if self._suspend or not self.is_real:
            if self.sim_comm is not None and t.is_cuda and not self._suspend:
                self._sim_wait(n * t.numel() * t.element_size())
            return torch.cat([t] * n) if n > 1 else t
        t = t.contiguous()
        out = torch.empty((n * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if self._native_ok(t):
            self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), self._code(t),
                                 torch.cuda.current_stream().cuda_stream)
        elif t.is_cuda and self.host_staged:
            self._no_capture()
            h = torch.empty((n * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype)
            dist.all_gather_into_tensor(h, t.cpu(), group=self.group)
            out.copy_(h)
        else:
            dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.is_real and self._native_ok(t):
            if not t.is_contiguous():
                raise ValueError("broadcast needs a contiguous tensor")
            self.comm.broadcast(t.data_ptr(), t.numel(), self._code(t), int(src), torch.cuda.current_stream().cuda_stream)
        elif self.is_real and t.is_cuda and self.host_staged:
            self._no_capture()
            h = t.cpu()
            dist.broadcast(h, src=self._global(src), group=self.group)
            t.copy_(h)
        elif self.is_real:
            dist.broadcast(t, src=self._global(src), group=self.group)
        return t

    def _global(self, r: int) -> int:
        """Global rank of group rank ``r`` (torch.distributed's src/dst are global ranks)."""
        return dist.get_global_rank(self.group, r) if self.group is not None and self.group != dist.group.WORLD \
            else r

    def broadcast_object(self, obj, src: int = 0):
        if not self.is_real:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=self._global(src), group=self.group)
        return box[0]

    def all_gather_object(self, obj) -> List:
        if not self.is_real:
            return [obj]
        out = [None] * dist.get_world_size(self.group)
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def barrier(self):
        if self.is_real:
            dist.barrier(group=self.group)

    # ------------------------------------------------------------ host-side agreement
    def _host_tensor_device(self):
        if self.comm is None and dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def all_reduce_int(self, v: int, op: str = "min") -> int:
        """Agree on one integer across ranks (``op`` = min | max | sum). Used for decisions every
        rank must take identically although each computes its own input (e.g. the KV pool size from
        its own free HBM: ranks that disagree would schedule differently and then deadlock in
        mismatched collectives)."""
        if not self.is_real:
            return int(v)
        t = torch.tensor([int(v)], dtype=torch.int64, device=self._host_tensor_device())
        rop = {"min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        return int(t.item())

    def agree(self, fn) -> Tuple[bool, str]:
        """Run ``fn()`` on every rank and agree on its success: ``(True, "")`` on every rank only if it raised
        on none. A rank where it raised (any Exception) reports ``(False, its error)``, the others
        ``(False, "")``, so all ranks take the same branch afterwards - a decision taken per rank (one rank
        eager, its peers in graphs) would leave the peers waiting in a collective the failed rank never joins."""
        err = ""
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - any failure (RuntimeError, HIP errors, OOM, ValueError) is agreed
            err = f"{type(e).__name__}: {e}"
        ok = self.all_reduce_int(0 if err else 1, "min")
        return bool(ok), err

    def check_consistent(self, what: str, fingerprint: dict) -> None:
        """Raise on every rank if any rank's ``fingerprint`` differs from rank 0's (a mismatched
        model / engine config would otherwise surface as a hang in the first diverging collective)."""
        if not self.is_real:
            return
        allfp = self.all_gather_object(fingerprint)
        bad = {r: {k: (fp.get(k), allfp[0].get(k)) for k in set(fp) | set(allfp[0]) if fp.get(k) != allfp[0].get(k)}
               for r, fp in enumerate(allfp) if fp != allfp[0]}
        if bad:
            raise RuntimeError(f"{what}: tensor-parallel ranks disagree (rank: {{key: (value, rank0 value)}}): {bad}")

    def close(self, abort: bool = False):
        """Release the native communicator (``abort``: without waiting for peers, e.g. after a failure)."""
        if self.comm is not None:
            self.comm.abort() if abort else self.comm.destroy()
            self.comm = None

    def __repr__(self):
        return f"TPGroup(rank={self.rank}, size={self.size}, {self.backend})"


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _pg_options(backend: str):
    """torch ``nccl`` process groups get the reference's high-priority internal stream (``dist.py:52-53``)."""
    if backend != "nccl" or not hasattr(dist, "ProcessGroupNCCL"):
        return None
    return dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)


def comm_mode() -> str:
    """Data plane on GPUs: 'native' (csrc/comm.cpp RcclComm, default) or 'torch' (torch's nccl process group)."""
    m = os.environ.get("LLMSS_COMM", "native")
    if m not in ("native", "torch"):
        raise ValueError(f"LLMSS_COMM must be 'native' or 'torch', not {m!r}")
    return m


def _rccl_comm(uid, nranks: int, rank: int, device: int):
    """One native communicator, created non-blocking with a deadline (csrc/comm.cpp RcclComm): a peer that never
    joins makes this rank abort and raise after ``LLMSS_RCCL_INIT_TIMEOUT_S`` (default 120 s) instead of blocking
    inside ncclCommInitRank forever (reference: the NCCL group's 60 s timeout, ``utils/dist.py:54,71``)."""
    from .. import _native

    timeout = float(os.environ.get("LLMSS_RCCL_INIT_TIMEOUT_S", "120"))
    return _native().RcclComm(uid, nranks, rank, device, timeout)


def _native_comm(rank: int, dp: int, tp: int, make_comm=None, unique_id=None):
    """One RCCL communicator per data-parallel replica (ranks r*tp .. r*tp+tp-1). Each replica leader draws a
    unique id; the ids travel over the CPU world group (every rank joins every broadcast), then each rank
    joins its replica's communicator and checks it with one all-reduce.

    Everything that can fail before the communicator init (drawing the id, the device) is agreed over gloo
    first, so a rank that fails there makes every rank raise instead of leaving its peers inside the init. The
    init itself is bounded (:func:`_rccl_comm`): a peer that never arrives - it died, or failed after the
    agreement - makes the waiting ranks abort their half-built communicator and raise at the deadline; the
    caller then agrees on the failure over gloo. ``make_comm`` / ``unique_id`` replace the native constructor and
    ncclGetUniqueId (CPU tests of this protocol)."""
    import time

    make_comm = make_comm or _rccl_comm
    if unique_id is None:
        from .. import _native

        unique_id = _native().rccl_unique_id
    uids, err = [], ""
    for r in range(dp):
        box = [None]
        if rank == r * tp:
            try:
                box = [unique_id()]
            except Exception as e:  # noqa: BLE001 - agreed below; the broadcast still runs
                err = f"ncclGetUniqueId: {e}"
        dist.broadcast_object_list(box, src=r * tp)
        uids.append(box[0])
    dev = 0
    try:
        dev = torch.cuda.current_device()
        torch.cuda.set_device(dev)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        err = err or f"device: {e}"
    r = rank // tp
    if uids[r] is None:
        err = err or "no unique id from the replica leader"
    ok = torch.tensor([0 if err else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok[0]):
        raise RuntimeError(f"rank {rank}: RCCL pre-init check failed ({err or 'on a peer'})")
    if os.environ.get("LLMSS_FAULT_INJECT", "") == f"{rank}:rccl_init:skip":  # tests: passes the agreement, then
        raise RuntimeError("injected: rank skipped the communicator init")  # never joins the init (dead peer)
    t0 = time.perf_counter()
    comm = make_comm(uids[r], tp, rank - r * tp, dev)
    COMM_INIT_INFO.update({"init_s": round(time.perf_counter() - t0, 3),
                           "timeout_s": float(os.environ.get("LLMSS_RCCL_INIT_TIMEOUT_S", "120"))})
    if not torch.cuda.is_available():  # protocol tests: no device self-check
        return comm
    from .. import _native

    C = _native()
    t = torch.full((4,), float(rank - r * tp + 1), dtype=torch.float32, device="cuda")
    comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), C.rccl_dtypes["float32"],
                    torch.cuda.current_stream().cuda_stream)
    want = tp * (tp + 1) / 2
    got = t.cpu()
    if not bool((got == want).all()):
        comm.abort()
        raise RuntimeError(f"rank {rank}: RCCL self-check all-reduce returned {got.tolist()}, expected {want}")
    COMM_INIT_INFO["first_collective_s"] = round(time.perf_counter() - t0 - COMM_INIT_INFO["init_s"], 3)
    return comm


COMM_INIT_INFO: dict = {}  # this rank's communicator set-up times (bench.py's runtime record)


# RCCL settings the decode all-reduce is timed under at start-up (LLMSS_RCCL_TUNE): the library's choice, then
# each protocol forced (RCCL reads NCCL_PROTO / NCCL_ALGO while it builds a communicator's tuning tables, so a
# communicator created under the variable keeps it). Each entry: (name, env overrides).
RCCL_CANDIDATES = [("default", {}), ("LL", {"NCCL_PROTO": "LL"}), ("LL128", {"NCCL_PROTO": "LL128"}),
                   ("Simple", {"NCCL_PROTO": "Simple"}), ("Tree", {"NCCL_ALGO": "Tree"})]
RCCL_TUNE_INFO: dict = {}  # what the start-up probe measured and kept (bench.py's runtime record)


def _time_all_reduce(comm, nbytes: int, reps: int = 20) -> float:
    """Microseconds per bf16 all-reduce of ``nbytes``, replayed from a HIP graph (as the decode graphs run it)."""
    from .. import _native

    code = _native().rccl_dtypes["bfloat16"]
    x = torch.ones(nbytes // 2, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            comm.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), code, s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            comm.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), code, torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    del g
    return best


def _agreed(fn, group=None):
    """Run ``fn()`` on every rank of ``group`` and agree on success (min over gloo): ``(True, result)`` only if
    it raised on no rank, so every rank takes the same branch of the probe below."""
    out, err = None, ""
    try:
        out = fn()
    except Exception as e:  # noqa: BLE001 - reported collectively
        err = str(e) or repr(e)
    ok = torch.tensor([0 if err else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if err:
        log.warning("rank %d: RCCL probe step failed: %s", dist.get_rank(), err)
    return bool(int(ok[0])), out


def _check_all_reduce(comm, tp: int, rank: int):
    """A candidate communicator must sum correctly before it may win: rank r contributes r + 1."""
    from .. import _native

    t = torch.full((1024,), float(rank + 1), dtype=torch.float32, device="cuda")
    comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _native().rccl_dtypes["float32"],
                    torch.cuda.current_stream().cuda_stream)
    want = tp * (tp + 1) / 2
    if not bool((t.cpu() == want).all()):
        raise RuntimeError(f"candidate all-reduce returned a wrong sum (expected {want})")


def _tune_native_comm(comm, rank: int, tp: int, nbytes: int, group=None, make_comm=None):
    """Start-up probe of the RCCL protocol / algorithm for the decode all-reduce (``nbytes``, the bench's 64
    sequences per GPU x hidden 4096 x bf16 at TP=8 = 4 MiB by default, LLMSS_RCCL_TUNE_BYTES). Opt-in
    (``LLMSS_RCCL_TUNE=1``) until it has run on a multi-GPU node. Every candidate of
    RCCL_CANDIDATES gets a communicator built under its environment (bounded init), must sum correctly on a
    fresh buffer, and has its graph-replayed all-reduce timed on every rank; each of these steps is agreed over
    gloo, so a step that fails on one rank drops the candidate on all of them (no rank leaves the probe's
    collective sequence alone). The max over ranks decides, all ranks keep the same setting, and a candidate
    must beat the library default by 5 %. Single replica (dp == 1) only: probe unique ids go over the world
    group."""
    from .. import _native

    C = _native()
    make_comm = make_comm or _rccl_comm
    dev = torch.cuda.current_device()
    ok, t = _agreed(lambda: _time_all_reduce(comm, nbytes), group)
    if not ok:
        return comm
    times, comms = {"default": t}, {"default": comm}
    saved = {k: os.environ.get(k) for _, env in RCCL_CANDIDATES for k in env}

    def restore():
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for name, env in RCCL_CANDIDATES[1:]:
            ok, uid = _agreed(lambda: C.rccl_unique_id() if rank == 0 else b"", group)
            if not ok:
                times[name] = None
                continue
            box = [uid]
            dist.broadcast_object_list(box, src=0, group=group)
            os.environ.update(env)
            try:
                ok, c = _agreed(lambda: make_comm(box[0], tp, rank, dev), group)
            finally:
                restore()
            if ok:
                ok, t = _agreed(lambda: (_check_all_reduce(c, tp, rank), _time_all_reduce(c, nbytes))[1], group)
            if not ok:
                if c is not None:
                    c.abort()
                times[name] = None
                continue
            times[name], comms[name] = t, c
    finally:
        restore()
    allt = [None] * dist.get_world_size(group)
    dist.all_gather_object(allt, times, group=group)
    worst = {n: (None if any(t.get(n) is None for t in allt) else max(t[n] for t in allt)) for n in times}
    okt = {n: v for n, v in worst.items() if v is not None}
    best = min(okt, key=lambda n: okt[n] if n == "default" else okt[n] / 0.95)
    for n, c in comms.items():
        if n != best:
            c.destroy()
    RCCL_TUNE_INFO.clear()
    RCCL_TUNE_INFO.update({"bytes": nbytes, "us": {n: (round(v, 2) if v is not None else None)
                                                   for n, v in worst.items()}, "kept": best,
                           "env": dict(dict(RCCL_CANDIDATES)[best])})
    if best != "default":  # later communicators of this process (none today) inherit the setting too
        os.environ.update(dict(RCCL_CANDIDATES)[best])
    log.info("rank %d: RCCL all-reduce %d KiB per setting (us, max over ranks): %s -> keeping %s", rank,
             nbytes >> 10, RCCL_TUNE_INFO["us"], best)
    return comms[best]


def initialize_distributed(timeout_s: Optional[int] = None, backend: Optional[str] = None, dp: Optional[int] = None):
    """Initialise torch.distributed from torchrun env vars.

    Returns ``(tp_group, rank, world_size)`` like the reference
    (``dist.py:40``); ``tp_group`` is a :class:`TPGroup`.

    On GPUs (``backend`` None) the torch process group is CPU-only (gloo: bootstrap, control plane,
    barriers) and the tensor data plane is a native RCCL communicator per replica (:func:`comm_mode`).
    ``backend="gloo"`` on GPUs stages device tensors through the host (several ranks sharing one GPU in
    tests); ``backend="nccl"`` / ``LLMSS_COMM=torch`` uses torch's RCCL process group for the data plane.

    ``dp`` (or ``LLMSS_DP``) > 1 splits the world into ``dp`` data-parallel replicas of
    ``world / dp`` consecutive ranks each (one node: a replica's ranks share an xGMI island). Every
    replica gets its own data-plane communicator and its own gloo control group;
    the returned TPGroup is this rank's replica (``.replica``, ``.dp``, ``.global_rank``).
    """
    if timeout_s is None:  # engine start-up (weight load, per-rank GEMM autotuning) runs between collectives
        timeout_s = _env_int("LLMSS_DIST_TIMEOUT_S", 600)
    rank = _env_int("RANK", 0)
    world_size = _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", rank)

    use_cuda = torch.cuda.is_available()
    if use_cuda:
        n = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % n)
    native = use_cuda and backend is None and comm_mode() == "native"
    if backend is None:
        backend = "nccl" if use_cuda and not native else "gloo"

    dp = int(dp if dp is not None else _env_int("LLMSS_DP", 1))
    if dp < 1 or world_size % dp:
        raise ValueError(f"data-parallel degree {dp} does not divide world size {world_size}")
    if world_size == 1:
        return TPGroup(0, 1), rank, world_size
    if os.environ.get("DEBUG") == "1":
        log.warning("DEBUG=1: fake process group, no collectives (numerically wrong by design)")
        return TPGroup(rank, world_size, fake=True), rank, world_size

    if not dist.is_initialized():
        if backend == "nccl":  # a hung or dead peer aborts the communicator after `timeout_s` (clean error, no hang)
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kwargs = dict(backend=backend, world_size=world_size, rank=rank, timeout=timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", torch.cuda.current_device())
            kwargs["pg_options"] = _pg_options(backend)
        dist.init_process_group(**kwargs)
    tp = world_size // dp
    comm, err = None, ""
    if native and tp > 1:
        try:
            comm = _native_comm(rank, dp, tp)
        except Exception as e:  # noqa: BLE001 - decided collectively below
            err = str(e)
        ok = torch.tensor([0 if err else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # CPU (gloo) world group: every rank takes the same path
        if int(ok[0]) and dp == 1 and os.environ.get("LLMSS_RCCL_TUNE", "0") == "1":
            try:
                comm = _tune_native_comm(comm, rank, tp, _env_int("LLMSS_RCCL_TUNE_BYTES", 4 << 20))
            except Exception as e:  # noqa: BLE001 - a failed probe keeps the library default
                log.warning("rank %d: RCCL setting probe failed (%s); keeping the default", rank, e)
        if not int(ok[0]):
            if comm is not None:
                comm.abort()
                comm = None
            if dp != 1:
                raise RuntimeError(f"rank {rank}: native RCCL communicator failed ({err or 'on a peer'})")
            # one replica: fall back to torch's RCCL process group for the data plane (same library, c10d's
            # bootstrap and stream handling) instead of failing the run
            log.warning("rank %d: native RCCL communicator failed (%s); data plane on torch's nccl group",
                        rank, err or "on a peer")
            data = dist.new_group(list(range(world_size)), backend="nccl", pg_options=_pg_options("nccl"))
            return TPGroup(rank, world_size, group=data), rank, world_size
    log.info("rank %d/%d initialised: process group %s, data plane %s", rank, world_size, backend,
             "native RCCL" if comm is not None else backend)
    if dp == 1:
        return TPGroup(rank, world_size, group=dist.group.WORLD, comm=comm), rank, world_size
    # the replica's control group carries the serving driver's leader heartbeat: its timeout is the
    # follower's leader timeout (EngineDriver.leader_timeout_s), not the long start-up timeout above
    ctrl_timeout = _env_int("LLMSS_LEADER_TIMEOUT_S", 300)
    mine = None
    for r in range(dp):  # new_group is collective over the world: every rank creates every group
        ranks = list(range(r * tp, (r + 1) * tp))
        data = dist.new_group(ranks, backend=backend, pg_options=_pg_options(backend)) if tp > 1 else None
        ctrl = dist.new_group(ranks, backend="gloo", timeout=timedelta(seconds=ctrl_timeout)) if tp > 1 else None
        if rank in ranks:
            mine = (r, data, ctrl)
    r, data, ctrl = mine
    g = TPGroup(rank - r * tp, tp, group=data, comm=comm)
    g.replica, g.dp, g.global_rank, g.ctrl_group = r, dp, rank, ctrl
    log.info("rank %d: data-parallel replica %d/%d, tensor-parallel rank %d/%d", rank, r, dp, g.rank, tp)
    return g, rank, world_size


class FakeBarrier:
    """Reference ``FakeBarrier`` (``dist.py:9-11``): the completed "work" a FakeGroup collective returns."""

    def wait(self):
        pass


class FakeGroup:
    """Reference ``FakeGroup(rank, size)`` (``dist.py:14-37``): the process group ``world_size == 1`` (or
    ``DEBUG=1``) code paths get. Collectives are no-ops, ``allgather`` copies the local tensor into the single
    output slot, ``size()`` / ``rank()`` report the constructor arguments. Anything in this package that takes
    a process group accepts one (:func:`as_tp_group` turns it into a :class:`TPGroup`: identity collectives at
    size 1, the fake no-communication mode above)."""

    def __init__(self, rank: int, size: int):
        self._rank = int(rank)
        self._size = int(size)

    def allreduce(self, *args, **kwargs):
        return FakeBarrier()

    def allgather(self, inputs, local_tensor, **kwargs):
        if not (len(inputs[0]) == len(local_tensor) == 1):
            raise ValueError(f"{len(inputs[0])} != {len(local_tensor)} != 1: FakeGroup joins single tensors")
        for inp in inputs:
            inp[0].data = local_tensor[0].data
        return FakeBarrier()

    def barrier(self, *args, **kwargs):
        return FakeBarrier()

    def size(self) -> int:
        return self._size

    def rank(self) -> int:
        return self._rank

    def __repr__(self):
        return f"FakeGroup(rank={self._rank}, size={self._size})"


# TPGroups created by initialize_torch_distributed for the torch ProcessGroup it hands out, so that code which
# passes that ProcessGroup back (Weights(..., process_group=pg)) runs on the same native communicator
_TP_FOR_PG = {}


def as_tp_group(group) -> TPGroup:
    """The :class:`TPGroup` for whatever a caller passes as a process group: a TPGroup itself, a reference
    :class:`FakeGroup` (size 1: identity collectives; size > 1: DEBUG-style fake, no communication), a torch
    ``ProcessGroup`` (the TPGroup initialize_torch_distributed built for it, else one over torch's collectives),
    or None (single process)."""
    if group is None:
        return TPGroup()
    if isinstance(group, TPGroup):
        return group
    if isinstance(group, FakeGroup):
        return TPGroup(group.rank(), group.size(), fake=group.size() > 1)
    tp = _TP_FOR_PG.get(id(group))
    if tp is not None and tp[0] is group:
        return tp[1]
    return TPGroup(group.rank(), group.size(), group=group)


def initialize_torch_distributed():
    """Reference-compatible ``initialize_torch_distributed() -> (process_group, rank, world_size)``
    (``dist.py:40-77``): a :class:`FakeGroup` at ``world_size == 1`` or ``DEBUG=1``, otherwise the default
    (world) torch ProcessGroup - so ``torch.distributed.barrier(process_group)`` works as in the reference's
    ``generate.py:62`` - after :func:`initialize_distributed` has set up the native data plane, which
    ``as_tp_group(process_group)`` (and so ``Weights`` / ``MODEL_REGISTRY``) picks up again. Unlike the reference
    the default process group exists at ``world_size == 1`` too when torch.distributed is used at all later
    (un-grouped ``dist.broadcast`` in the reference's single-GPU generate.py raises): here callers get
    a FakeGroup and no default group, exactly like the reference, so use the returned group."""
    tp, rank, world_size = initialize_distributed()
    if world_size == 1 or tp.fake:
        return FakeGroup(rank, world_size), rank, world_size
    if tp.dp > 1:
        # data-parallel replicas (LLMSS_DP): this rank's replica, not the world, is the tensor-parallel group -
        # its CPU control group stands in for the process group (WORLD would shard the model
        # over every replica's ranks)
        if tp.size == 1:
            return FakeGroup(0, 1), rank, world_size
        pg = tp.ctrl_group
    else:
        pg = dist.group.WORLD
    _TP_FOR_PG[id(pg)] = (pg, tp)
    return pg, rank, world_size
