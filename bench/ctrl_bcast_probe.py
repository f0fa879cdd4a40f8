"""Cost of the serving driver's per-step control record (serving/driver.py EngineDriver._bcast) at 2 / 4 / 8
ranks, over either channel:
  gloo: a 16-byte header broadcast over the CPU control group (+ the pickled payload when there is one);
  shm:  the native shared-memory ring (csrc/ctrl.cpp CtrlRing): a 1-byte record, or the payload record.

Runs on the CPU (as on one node). Prints one JSON line per (world size, mode) with the median / p99
microseconds per step on the leader and on the slowest follower, with no payload and with a pickled
admission of 8 requests every 16 steps.

usage: python bench/ctrl_bcast_probe.py [--ranks 2 4 8] [--steps 2000] [--ctrl gloo shm]
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, ctrl, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hdr = torch.zeros(2, dtype=torch.int64)
    payload = pickle.dumps({"new": [(i, list(range(128)), {"max_new_tokens": 128}) for i in range(8)], "abort": []})
    ring = None
    if ctrl == "shm":
        from llmss_amd import _native

        C = _native()
        name = [f"/llmss_probe_{os.getpid()}"]
        dist.broadcast_object_list(name, src=0)
        if rank == 0:
            ring = C.CtrlRing(name[0], True, 1 << 24, world - 1, 0)
        dist.barrier()
        if rank:
            ring = C.CtrlRing(name[0], False, 0, 0, rank - 1)
        if rank == 0:
            assert ring.wait_attached(60.0)
    for mode in ("header", "header+payload/16"):
        dist.barrier()
        ts = []
        for s in range(steps):
            t = time.perf_counter()
            with_payload = mode != "header" and s % 16 == 0
            if ring is not None:
                if rank == 0:
                    ring.send(b"\x02" + payload if with_payload else b"\x00", 60.0)
                else:
                    rec = ring.recv(60.0)
                    if rec[:1] == b"\x02":
                        pickle.loads(rec[1:])
            else:
                hdr[0] = len(payload) if (rank == 0 and with_payload) else 0
                dist.broadcast(hdr, src=0)
                n = int(hdr[0])
                if n:
                    buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if rank == 0 else torch.empty(n, dtype=torch.uint8)
                    dist.broadcast(buf, src=0)
                    if rank:
                        pickle.loads(buf.numpy().tobytes())
            ts.append(time.perf_counter() - t)
        ts = np.array(ts[100:]) * 1e6
        q.put((mode, rank, float(np.median(ts)), float(np.percentile(ts, 99))))
    # one-way latency with the leader busy 3 ms per step (an engine step) before it sends: the time from
    # the leader's send to the follower holding the record (CLOCK_MONOTONIC is shared by the processes)
    dist.barrier()
    lat = []
    ts_t = torch.zeros(1, dtype=torch.float64)
    for s in range(min(steps, 400)):
        if rank == 0:
            time.sleep(0.003)
            t = time.perf_counter()
            if ring is not None:
                ring.send(b"\x00" + pickle.dumps(t), 60.0)
            else:
                ts_t[0] = t
                dist.broadcast(ts_t, src=0)
        else:
            if ring is not None:
                t = pickle.loads(ring.recv(60.0)[1:])
            else:
                dist.broadcast(ts_t, src=0)
                t = float(ts_t[0])
            lat.append(time.perf_counter() - t)
    if rank:
        lat = np.array(lat[20:]) * 1e6
        q.put(("one-way@3ms", rank, float(np.median(lat)), float(np.percentile(lat, 99))))
    else:
        q.put(("one-way@3ms", 0, 0.0, 0.0))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--ctrl", nargs="+", default=["gloo", "shm"])
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    for ctrl in a.ctrl:
        for w in a.ranks:
            q = ctx.Queue()
            port = _port()
            procs = [ctx.Process(target=_worker, args=(r, w, port, a.steps, ctrl, q)) for r in range(w)]
            for p in procs:
                p.start()
            res = [q.get(timeout=600) for _ in range(3 * w)]
            for mode in ("header", "header+payload/16", "one-way@3ms"):
                lead = [r for r in res if r[0] == mode and r[1] == 0][0]
                fol = [r for r in res if r[0] == mode and r[1] > 0]
                print(json.dumps({"ctrl": ctrl, "ranks": w, "mode": mode,
                                  "leader_p50_us": round(lead[2], 1), "leader_p99_us": round(lead[3], 1),
                                  "follower_p50_us": round(max(r[2] for r in fol), 1),
                                  "follower_p99_us": round(max(r[3] for r in fol), 1)}), flush=True)
            for p in procs:
                p.join(60)


if __name__ == "__main__":
    sys.exit(main())
