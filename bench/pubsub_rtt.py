"""Pub/sub turnaround without a GPU: how long a cohort of closed-loop clients' re-submissions take to get back
to the engine through gRPC front-end -> RESP broker -> consumer (the spread that splits GPT-2-XL's batches into
cohorts, profiles/r6_pubsub).

A stand-in engine completes every request submitted so far in one "step" (as a decode step ends a cohort) and
records when each next request arrives; the clients are closed-loop gRPC threads in their own process, the
front-end and broker in a third (bench/serving_bench.py --frontend), as in `serving_bench.py --mode pubsub`.
Prints one JSON line: per round, the time from the cohort's completion to its last re-submission (p50 / max).

usage: python bench/pubsub_rtt.py [--clients 64] [--rounds 20]
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HERE = os.path.dirname(os.path.abspath(__file__))


class _Handle:
    def __init__(self, ids, rid):
        self.rid = rid
        self.output_ids = list(ids[:8])
        self.finish_reason = "length"
        self.metrics = {"ttft_s": 0.001, "e2e_s": 0.002}
        self.error = ""
        self.done = threading.Event()


class FakeDriver:
    """EngineDriver stand-in: submissions queue up; complete() finishes all of them at once."""
    leader = True

    def __init__(self):
        self.mu = threading.Lock()
        self.pending = []
        self.arrivals = []

    def submit(self, ids, params, on_done=None, on_token=None, **_):
        with self.mu:
            h = _Handle(ids, len(self.arrivals))
            self.pending.append((h, on_done))
            self.arrivals.append(time.perf_counter())
        return h

    def abort(self, rid):
        pass

    def complete(self):
        with self.mu:
            done, self.pending = self.pending, []
        t = time.perf_counter()
        for h, cb in done:
            h.done.set()
            cb(h)
        return t, len(done)


def clients(port, n, rounds, broker_port=0):
    import concurrent.futures as cf

    import grpc

    from llmss_amd.serving.grpc_api import GenerateRequest, Stub

    def one_broker(i):  # --direct-broker: LPUSH + BRPOP on the broker itself, no gRPC front-end
        from llmss_amd.serving.broker import PQUEUE, RedisBroker, reply_key

        b = RedisBroker("127.0.0.1", broker_port)
        for r in range(rounds):
            rid = f"c{i}r{r}"
            b.lpush(PQUEUE, json.dumps({"prompt": "x" * 128, "max_new_tokens": 8, "request_id": rid}))
            b.brpop(reply_key(rid), 60)

    def one(i):
        if broker_port:
            return one_broker(i)
        with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
            stub = Stub(ch)
            for r in range(rounds):
                stub.Generate(GenerateRequest(prompt="x" * 128, max_new_tokens=8, request_id=f"c{i}r{r}"), timeout=60)

    with cf.ThreadPoolExecutor(n) as ex:
        list(ex.map(one, range(n)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--client-port", type=int, default=0)
    ap.add_argument("--direct-broker", action="store_true", help="clients talk RESP to the broker (no gRPC hop)")
    ap.add_argument("--direct-grpc", action="store_true", help="clients on the engine's own gRPC service (no broker)")
    ap.add_argument("--broker-port", type=int, default=0, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.client_port:
        return clients(a.client_port, a.clients, a.rounds, a.broker_port)
    from llmss_amd.serving.broker import RedisBroker
    from llmss_amd.serving.consumer import Consumer
    from llmss_amd.utils.tokenizer import ByteTokenizer

    fe = subprocess.Popen([sys.executable, os.path.join(HERE, "serving_bench.py"), "--frontend"], stdin=subprocess.PIPE,
                          stdout=subprocess.PIPE, text=True)
    broker_port, grpc_port = map(int, fe.stdout.readline().split())
    drv = FakeDriver()
    consumer = Consumer(drv, ByteTokenizer(), RedisBroker("127.0.0.1", broker_port), poll_timeout=0.05).start()
    if a.direct_grpc:
        from llmss_amd.serving.grpc_api import EngineServicer, serve

        srv = serve(EngineServicer(drv, ByteTokenizer()), port=0, host="127.0.0.1")
        grpc_port = srv.bound_port
    cl = subprocess.Popen([sys.executable, os.path.abspath(__file__), f"--client-port={grpc_port}",
                           f"--clients={a.clients}", f"--rounds={a.rounds}"]
                          + ([f"--broker-port={broker_port}"] if a.direct_broker else []))
    spreads = []
    try:
        for r in range(a.rounds):
            deadline = time.time() + 60
            while True:  # the whole cohort is in
                with drv.mu:
                    n = len(drv.pending)
                if n >= a.clients or time.time() > deadline:
                    break
                time.sleep(0.0005)
            if r:
                with drv.mu:
                    last = max(drv.arrivals[-a.clients:])
                spreads.append(last - t_done)
            time.sleep(0.005)  # "prefill + decode"
            t_done, _ = drv.complete()
            with drv.mu:
                drv.arrivals.clear()
        cl.wait(60)
    finally:
        consumer.stop()
        fe.stdin.close()
        fe.wait(30)
    spreads.sort()
    print(json.dumps({"metric": "pubsub_cohort_turnaround_ms", "clients": a.clients, "rounds": len(spreads),
                      "path": "resp" if a.direct_broker else ("direct grpc" if a.direct_grpc else "grpc front-end"),
                      "p50_ms": round(spreads[len(spreads) // 2] * 1e3, 2), "max_ms": round(spreads[-1] * 1e3, 2)}))


if __name__ == "__main__":
    main()
