"""Serving soak on one GPU: a model (random init) behind the in-process gRPC Generate service, driven for --seconds by
--clients threads with mixed traffic - prompts of 1-600 tokens, 1-200 new tokens, greedy and sampled, unary and
streaming calls, a share of streams cancelled part-way and a share of unary calls whose deadline expires. Checks:
every completed call returned exactly its max_new_tokens (ignore_eos); only the expected errors occurred; at the end
the engine is idle with every KV block back in the pool and the driver healthy; and one greedy probe request, run
alone before and after the load, returns the same tokens (nothing leaks from one request into another).

--pubsub: the same traffic through the pub/sub path instead (gRPC front-end -> embedded broker -> consumer ->
engine); then also every broker list must be gone at the end (acknowledged, popped or expired by its TTL).

usage: python bench/soak.py [--model gpt2-xl] [--seconds 120] [--clients 48] [--pubsub]
"""
import argparse
import collections
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--clients", type=int, default=48)
    ap.add_argument("--pubsub", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="fp8 (e4m3) weights: W8A8 / MX-fp8 GEMMs")
    ap.add_argument("--device", default="cuda", help="cuda, or cpu for a dry run of the harness on a tiny preset")
    a = ap.parse_args()

    import grpc

    from llmss_amd.engine import LLMEngine, build_model
    from llmss_amd.serving.driver import EngineDriver
    from llmss_amd.serving.grpc_api import EngineServicer, GenerateRequest, Stub, serve
    from llmss_amd.utils.tokenizer import load_tokenizer

    dev = torch.device("cuda", 0) if a.device == "cuda" else torch.device("cpu")
    model = build_model(a.model, None, "bf16" if a.device == "cuda" else "fp32", dev, random_init=True, fp8=a.fp8)
    V = model.cfg.vocab_size
    eng = LLMEngine(model, max_num_seqs=64, max_batched_tokens=8192, max_model_len=1024)
    free0 = eng.sched.num_free_blocks()
    drv = EngineDriver(eng).start()
    tok = load_tokenizer(a.model, V)
    broker = consumer = None
    if a.pubsub:
        from llmss_amd.serving.broker import MiniRedisServer, RedisBroker
        from llmss_amd.serving.consumer import Consumer
        from llmss_amd.serving.grpc_api import AioBrokerServicer

        broker = MiniRedisServer().start()
        consumer = Consumer(drv, tok, RedisBroker(broker.host, broker.port), reply_ttl_s=5).start()
        server = serve(AioBrokerServicer(broker.host, broker.port), port=0, host="127.0.0.1")
    else:
        server = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
    ch = grpc.insecure_channel(f"127.0.0.1:{server.bound_port}")
    stub = Stub(ch)
    probe = GenerateRequest(prompt_token_ids=list(range(7, 57)), max_new_tokens=32, is_greedy=True, ignore_eos=True)
    before = list(stub.Generate(probe, timeout=300).token_ids)

    stats = collections.Counter()
    bad = []
    lock = threading.Lock()
    t_end = time.time() + a.seconds

    def note(k, err=None):
        with lock:
            stats[k] += 1
            if err is not None and len(bad) < 20:
                bad.append(err)

    def client(ci):
        rng = np.random.default_rng(1000 + ci)
        while time.time() < t_end:
            n, g = int(rng.integers(1, 601)), int(rng.integers(1, 201))
            req = GenerateRequest(prompt_token_ids=rng.integers(0, V, n).tolist(), max_new_tokens=g,
                                  is_greedy=bool(rng.random() < 0.3), temperature=1.0, top_p=0.95,
                                  top_k=int(rng.choice([0, 50])), seed=int(rng.integers(1, 1 << 30)), ignore_eos=True)
            kind = rng.random()
            try:
                if kind < 0.55:
                    r = stub.Generate(req, timeout=300)
                    ok = len(r.token_ids) == g and r.finish_reason == "length"
                    note("unary_ok" if ok else "unary_wrong", None if ok else ("unary", n, g, len(r.token_ids),
                                                                               r.finish_reason))
                elif kind < 0.75:
                    toks = [t for t in stub.GenerateStream(req, timeout=300)]
                    ok = len(toks) == g + 1 and toks[-1].finished and all(t.token_id >= 0 for t in toks[:-1])
                    note("stream_ok" if ok else "stream_wrong", None if ok else ("stream", n, g, len(toks)))
                elif kind < 0.9:
                    call = stub.GenerateStream(req, timeout=300)
                    stop_at = int(rng.integers(0, max(1, g // 2)))
                    got = 0
                    for _ in call:
                        got += 1
                        if got > stop_at:
                            call.cancel()
                            break
                    note("stream_cancelled")
                else:
                    r = stub.Generate(req, timeout=float(rng.uniform(0.02, 0.5)))
                    ok = len(r.token_ids) == g
                    note("deadline_met" if ok else "deadline_wrong", None if ok else ("deadline", n, g))
            except grpc.RpcError as e:
                code = e.code()
                if code in (grpc.StatusCode.DEADLINE_EXCEEDED, grpc.StatusCode.CANCELLED):
                    note("expected_" + code.name.lower())
                else:
                    note("rpc_error", (code.name, e.details()))

    ths = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(a.clients)]
    t0 = time.time()
    for t in ths:
        t.start()
    last = t0
    while any(t.is_alive() for t in ths):
        time.sleep(1.0)
        if time.time() - last > 20:
            last = time.time()
            print(f"[soak] {time.time() - t0:.0f}s {dict(stats)} tokens={eng.stats['tokens']}", file=sys.stderr,
                  flush=True)
    for t in ths:
        t.join(300)
    # idle: every request finished or aborted, every KV block back in the pool
    deadline = time.time() + 120
    while time.time() < deadline and (drv.handles or eng.sched.num_running() or eng.sched.num_waiting()):
        time.sleep(0.2)
    idle = not drv.handles and not eng.sched.num_running() and not eng.sched.num_waiting()
    left_keys = None
    if broker is not None:  # abandoned replies expire (TTL 5 s); acknowledged requests leave no processing entry
        time.sleep(7)
        left_keys = sorted(broker._lists)[:20]  # the consumer's polls keep the broker's once-a-second sweep running
    free1 = eng.sched.num_free_blocks()
    after = list(stub.Generate(probe, timeout=300).token_ids)
    out = {"model": a.model, "fp8": a.fp8, "path": "pubsub" if a.pubsub else "grpc", "seconds": round(time.time() - t0, 1), "clients": a.clients, "outcomes": dict(stats),
           "engine_tokens": eng.stats["tokens"], "engine_steps": eng.stats["steps"],
           "preemptions": eng.stats["preemptions"], "idle_at_end": idle, "free_blocks": [free0, free1],
           "probe_same": before == after, "driver_healthy": drv.error is None,
           "engine_requests_left": len(eng.requests), "broker_lists_left": left_keys, "errors": bad}
    ok = (idle and free1 == free0 and not left_keys and before == after and drv.error is None and not bad
          and stats["unary_ok"] > 0 and stats["stream_ok"] > 0)
    out["pass"] = ok
    print(json.dumps(out), flush=True)
    ch.close()  # the client channel's core threads end before the interpreter does
    server.stop(1).wait(30)
    if consumer is not None:
        consumer.stop()
        broker.stop()
    drv.stop()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
