"""Cross-stream dependency cost on MI355X (HIP graphs and eager): a compute stream of spin kernels with a side
stream whose kernel overlaps them, joined back with events - as the two-micro-batch decode schedule does.

usage: python bench/xq_probe.py [--us 20] [--side-us 10] [--n 16]
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--us", type=float, default=20.0)
    ap.add_argument("--side-us", type=float, default=10.0)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--arms", default="", help="comma list (default: all)")
    ap.add_argument("--modes", default="graph,eager")
    a = ap.parse_args()
    torch.cuda.init()
    torch.cuda._sleep(1000)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(2_000_000)
    e.record()
    e.synchronize()
    cyc = 2_000_000 / (s.elapsed_time(e) * 1e3)
    K = lambda: torch.cuda._sleep(int(a.us * cyc))
    C = lambda: torch.cuda._sleep(int(a.side_us * cyc))
    side = torch.cuda.Stream()

    def serial():
        cur = torch.cuda.current_stream()  # inside: the capture stream under torch.cuda.graph
        for _ in range(2 * a.n):
            K()

    def fork_join(lag):
        cur = torch.cuda.current_stream()  # inside: the capture stream under torch.cuda.graph
        evs = []
        for i in range(a.n):
            K()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                C()
                ev = torch.cuda.Event()
                ev.record(side)
            evs.append(ev)
            K()
            if len(evs) > lag:
                cur.wait_event(evs[-1 - lag])
        for ev in evs[-lag:] if lag else []:
            cur.wait_event(ev)
        cur.wait_stream(side)

    def fork_only():
        cur = torch.cuda.current_stream()  # inside: the capture stream under torch.cuda.graph  # side work never joined until the end: no wait packet on the compute stream inside
        for i in range(a.n):
            K()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                C()
            K()
        cur.wait_stream(side)

    def join_done():
        cur = torch.cuda.current_stream()  # inside: the capture stream under torch.cuda.graph  # the compute stream waits on an event that completed long before
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            C()
            ev = torch.cuda.Event()
            ev.record(side)
        for i in range(a.n):
            K()
            K()
            cur.wait_event(ev)

    def tbo(wait_first):
        cur = torch.cuda.current_stream()  # inside: the capture stream under torch.cuda.graph  # the two-micro-batch decode pattern: block j waits for its own previous side kernel
        pend = [None, None]
        for i in range(a.n):
            for j in (0, 1):
                if wait_first and pend[j] is not None:
                    cur.wait_event(pend[j])
                K()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    C()
                    ev = torch.cuda.Event()
                    ev.record(side)
                if not wait_first and pend[1 - j] is not None:
                    cur.wait_event(pend[1 - j])  # the other block's event, right after this block's fork
                pend[j] = ev
        cur.wait_stream(side)

    arms = {"tbo": lambda: tbo(True), "tbo_wait_after_fork": lambda: tbo(False), "serial": serial, "fork_join": lambda: fork_join(0), "fork_join_lag1": lambda: fork_join(1),
            "fork_only": fork_only, "join_done": join_done}
    out = {"kernel_us": a.us, "side_us": a.side_us, "n": a.n}
    if a.arms:
        arms = {k: v for k, v in arms.items() if k in a.arms.split(",")}
    for name, fn in arms.items():
        for mode in a.modes.split(","):
            fn()
            torch.cuda.synchronize()
            if mode == "graph":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fn()
                run = g.replay
            else:
                run = fn
            run()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(5):
                s.record()
                run()
                e.record()
                e.synchronize()
                best = min(best, s.elapsed_time(e) * 1e3)
            # per compute kernel: wall / (2 n) - kernel time = added cost per compute kernel
            out[f"{name}_{mode}_us"] = round(best, 1)
            nk = 2 * a.n
            out[f"{name}_{mode}_extra_per_kernel_us"] = round((best - nk * a.us) / nk, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
