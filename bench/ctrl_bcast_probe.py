"""Cost of the serving driver's per-step control header (serving/driver.py EngineDriver._bcast): one 16-byte
gloo broadcast from the leader over the CPU control group per engine step, at 2 / 4 / 8 ranks.

Runs on the CPU (gloo over loopback TCP, as on one node). Prints one JSON line per world size with the
median / p99 microseconds per header broadcast, and the same with a payload-bearing step (a pickled
admission of 8 requests) every 16 steps.

usage: python bench/ctrl_bcast_probe.py [--ranks 2 4 8] [--steps 2000]
"""
import argparse
import json
import os
import pickle
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hdr = torch.zeros(2, dtype=torch.int64)
    payload = pickle.dumps({"new": [(i, list(range(128)), {"max_new_tokens": 128}) for i in range(8)], "abort": []})
    for mode in ("header", "header+payload/16"):
        dist.barrier()
        ts = []
        for s in range(steps):
            t = time.perf_counter()
            with_payload = mode != "header" and s % 16 == 0
            hdr[0] = len(payload) if (rank == 0 and with_payload) else 0
            dist.broadcast(hdr, src=0)
            n = int(hdr[0])
            if n:
                buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if rank == 0 else torch.empty(n, dtype=torch.uint8)
                dist.broadcast(buf, src=0)
            ts.append(time.perf_counter() - t)
        if rank == 0:
            ts = np.array(ts[100:]) * 1e6
            q.put({"ranks": world, "mode": mode, "p50_us": round(float(np.median(ts)), 1),
                   "p99_us": round(float(np.percentile(ts, 99)), 1), "mean_us": round(float(ts.mean()), 1)})
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    for w in a.ranks:
        q = ctx.Queue()
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, w, port, a.steps, q)) for r in range(w)]
        for p in procs:
            p.start()
        for _ in range(2):
            print(json.dumps(q.get(timeout=600)), flush=True)
        for p in procs:
            p.join(60)


if __name__ == "__main__":
    sys.exit(main())
