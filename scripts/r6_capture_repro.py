"""Minimal reproduction of round 5's segfault in hipStreamEndCapture (profiles/r5_tbo/two_stream_capture_segfault.txt):
decode-graph capture with micro-batch B on a second compute stream, i.e. three streams (compute, compute2, comm)
joined by events. No model, no RCCL: small torch kernels stand in for the GEMMs and the collectives.

usage: python scripts/r6_capture_repro.py PATTERN     (one pattern per process: a segfault ends only that run)
patterns:
  two      compute + comm, fork/join by wait_stream (the in-tree _reduce_rows / _reduce_cols shape)
  events   compute + comm, per-chunk torch.cuda.Event recorded on comm, waited on by compute (_hidden_states_overlap)
  three    compute + compute2 + comm, every side stream joined back to the capturing stream before the end
  xalloc   three, and micro-batch B allocates on compute2 and frees the block before the join (allocator
           cross-stream free inside capture)
  unjoined three, with compute2's last work never joined back (the failure mode to rule in or out)
  late     three, with the final join done by waiting on an event recorded on compute2 BEFORE its last kernel
  pool     xalloc captured twice into two graphs that share one memory pool (the engine's per-bucket graphs)
  xcap     capture 1 records an event on the comm stream; capture 2 waits on that same event (an event recorded in
           one capture, waited on in another)
A "_rccl" suffix (two_rccl, three_rccl, ...) makes every comm-stream op a native RCCL all-reduce on a one-rank
communicator (csrc/comm.cpp RcclComm), as the engine's captured collectives are.
Prints one JSON line: pattern, result ("ok" or the Python exception), replay check.
"""
import json
import sys

import torch


def main():
    pat = sys.argv[1]
    rccl = pat.endswith("_rccl")
    pat = pat[:-5] if rccl else pat
    dev = torch.device("cuda", 0)
    comm_obj = None
    if rccl:
        sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
        from llmss_amd import _native

        C = _native()
        comm_obj = C.RcclComm(C.rccl_unique_id(), 1, 0, 0)
        code = C.rccl_dtypes["float32"]

    def reduce_(t):  # the "all-reduce" on the current (comm) stream
        if comm_obj is None:
            t.mul_(0.5)
        else:
            comm_obj.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), code, torch.cuda.current_stream().cuda_stream)
    cur = torch.cuda.Stream(device=dev)
    s2 = torch.cuda.Stream(device=dev)
    comm = torch.cuda.Stream(device=dev)
    x = torch.randn(256, 256, device=dev)
    w = torch.randn(256, 256, device=dev)
    outs = {}

    def body():
        a = x @ w  # micro-batch A on the capturing stream
        if pat in ("two", "events"):
            evs = []
            for c in range(4):
                y = a @ w
                comm.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(comm):
                    reduce_(y)
                    if pat == "events":
                        ev = torch.cuda.Event()
                        ev.record(comm)
                        evs.append(ev)
                outs[c] = y
            if pat == "events":
                for ev in evs:
                    torch.cuda.current_stream().wait_event(ev)
            else:
                torch.cuda.current_stream().wait_stream(comm)
            return
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):  # micro-batch B on a second compute stream
            b = x @ w
            if pat == "xalloc":
                tmp = b @ w
                b = b + tmp
                del tmp  # block freed on s2 while capturing
            b2 = b @ w
        comm.wait_stream(s2)
        with torch.cuda.stream(comm):
            reduce_(b2)
            ev_b = torch.cuda.Event()
            ev_b.record(comm)
        comm.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(comm):
            reduce_(a)
        if pat == "late":
            ev_early = torch.cuda.Event()
            ev_early.record(s2)
            with torch.cuda.stream(s2):
                b2.add_(1.0)  # work after the recorded event: never joined
            torch.cuda.current_stream().wait_event(ev_early)
        elif pat == "unjoined":
            with torch.cuda.stream(s2):
                b2.add_(1.0)
        else:
            torch.cuda.current_stream().wait_stream(s2)
        torch.cuda.current_stream().wait_event(ev_b)
        torch.cuda.current_stream().wait_stream(comm)
        outs["a"], outs["b"] = a, b2

    res = {"pattern": pat + ("_rccl" if rccl else "")}
    base = {"pool": "xalloc", "xcap": "three"}.get(pat, pat)
    with torch.cuda.stream(cur):
        pat, real = base, pat
        body()  # eager warm-up
        torch.cuda.synchronize()
        try:
            if real in ("pool", "xcap"):
                pool = torch.cuda.graph_pool_handle()
                g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                keep = torch.cuda.Event()
                with torch.cuda.graph(g1, pool=pool, capture_error_mode="thread_local"):
                    body()
                    if real == "xcap":
                        comm.wait_stream(torch.cuda.current_stream())
                        keep.record(comm)
                        torch.cuda.current_stream().wait_stream(comm)
                with torch.cuda.graph(g2, pool=pool, capture_error_mode="thread_local"):
                    if real == "xcap":
                        torch.cuda.current_stream().wait_event(keep)
                    body()
                g1.replay()
                g2.replay()
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    body()
                g.replay()
            torch.cuda.synchronize()
            res["result"] = "ok"
        except Exception as e:  # noqa: BLE001 - report what HIP said
            res["result"] = f"{type(e).__name__}: {str(e)[:300]}"
    print(json.dumps(res), flush=True)
    if comm_obj is not None:
        comm_obj.destroy()


if __name__ == "__main__":
    main()
