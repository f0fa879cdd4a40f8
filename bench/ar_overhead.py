"""Cost of a torch.distributed (RCCL) all-reduce inside a captured HIP graph, on one GPU (one-member
communicator): ProcessGroupNCCL runs every collective on its own internal stream, so each call in a
captured decode step is a fork to that stream and a join back - graph edges between streams.

usage: python bench/ar_overhead.py [--mib 4] [--iters 64]
Prints per-iteration microseconds of: a small kernel alone; the kernel + a dist.all_reduce; the kernel +
an all-reduce on a side stream joined back by events (what the bucketed overlap path records).
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_us(fn, iters, reps=5):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return best


def eager_us(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=64)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = int(a.mib * (1 << 20) // 2)
    x = torch.randn(n, device=dev).to(torch.bfloat16)
    y = torch.zeros(1 << 16, device=dev)
    side = torch.cuda.Stream(device=dev, priority=-1)

    def k():
        y.add_(1.0)

    def k_ar():
        y.add_(1.0)
        dist.all_reduce(x)

    def k_side():
        y.add_(1.0)
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            x.mul_(1.0)
        cur.wait_stream(side)

    res = {"mib": a.mib, "iters": a.iters}
    for name, fn in (("kernel", k), ("kernel+all_reduce", k_ar), ("kernel+side_stream_kernel", k_side)):
        res[f"{name}_graph_us"] = round(graph_us(fn, a.iters), 2)
        res[f"{name}_eager_us"] = round(eager_us(fn, a.iters), 2)
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
