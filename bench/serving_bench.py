"""Serving benchmark: concurrent gRPC clients against the engine (BASELINE: "GPT-2-XL TP=1 bf16 on
one MI355X served over gRPC"; "pubsub producer/consumer under concurrent gRPC clients").

  --mode grpc    clients -> gRPC Generate service on the engine driver (direct)
  --mode pubsub  clients -> gRPC front-end -> RESP broker (mini Redis) -> consumer -> engine
                 (front-end and broker in a process each, as a producer server and Redis would be;
                 --frontend-inproc puts them in the engine process, sharing its interpreter lock)

Random-init weights of the named architecture, random printable prompts (byte tokenizer: one
token per character). Prints one JSON line: output tokens/s over the timed requests, p50 request
latency and p50 server-side TTFT.

usage: python bench/serving_bench.py [--model gpt2-xl] [--mode grpc|pubsub] [--clients 64] [--requests 4]
       python bench/serving_bench.py --rate 20 --num-requests 256 --long-frac 0.1 --long-len 2048   (open loop)
Open loop compares scheduling policies: LLMSS_PREFILL_CHUNK=-1 (whole prompts) vs the default chunked prefill.
"""
import argparse
import concurrent.futures as cf
import faulthandler
import json
import os
import random
import string
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_clients(a):
    """Closed-loop clients: each thread sends `requests` requests back to back (one warmup first)."""
    import grpc

    from llmss_amd.serving.grpc_api import GenerateRequest, Stub

    rng = random.Random(0)
    alphabet = string.ascii_letters + string.digits + " "

    def client(i, n):
        out = []
        with grpc.insecure_channel(f"127.0.0.1:{a.client_port}") as ch:
            stub = Stub(ch)
            for r in range(n):
                prompt = "".join(rng.choice(alphabet) for _ in range(a.prompt_len))
                t0 = time.perf_counter()
                resp = stub.Generate(GenerateRequest(prompt=prompt, max_new_tokens=a.gen_len, temperature=1.0,
                                                     top_p=0.95, top_k=50, request_id=f"c{i}r{r}"), timeout=600)
                out.append((time.perf_counter() - t0, len(resp.token_ids), float(resp.ttft_s)))
        return out

    with cf.ThreadPoolExecutor(a.clients) as ex:  # warmup: one request per client
        list(ex.map(lambda i: client(i, 1), range(a.clients)))
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(a.clients) as ex:
        res = [x for r in ex.map(lambda i: client(i, a.requests), range(a.clients)) for x in r]
    el = time.perf_counter() - t0
    toks = sum(n for _, n, _ in res)
    lat = np.median([l for l, _, _ in res]) * 1e3
    ttft = np.median([t for _, _, t in res if t > 0] or [float("nan")]) * 1e3
    print(json.dumps({"metric": "serving_output_tokens_per_sec", "value": round(toks / el, 2), "unit": "tokens/s",
                      "clients": a.clients, "requests": len(res), "prompt_len": a.prompt_len, "gen_len": a.gen_len,
                      "p50_request_latency_ms": round(float(lat), 2), "p50_ttft_ms": round(float(ttft), 2),
                      "wall_s": round(el, 3)}), flush=True)


def run_open_loop(a):
    """Open-loop arrivals: `num_requests` requests at Poisson times of mean rate `rate` req/s, each streamed
    (GenerateStream) so every token's arrival is timed on the client. A `long_frac` share of the prompts is
    `long_len` characters long (the prompts that stall running decodes unless prefill is chunked).
    Reports p50 / p99 of TTFT, of each request's mean time per output token, and of the worst gap
    between two consecutive tokens of a request."""
    import threading

    import grpc

    from llmss_amd.serving.grpc_api import GenerateRequest, Stub

    rng = random.Random(0)
    alphabet = string.ascii_letters + string.digits + " "
    plan, t = [], 0.0
    for i in range(a.num_requests):
        t += rng.expovariate(a.rate)
        n = a.long_len if rng.random() < a.long_frac else a.prompt_len
        plan.append((t, "".join(rng.choice(alphabet) for _ in range(n))))
    res = [None] * len(plan)
    ch = grpc.insecure_channel(f"127.0.0.1:{a.client_port}")
    stub = Stub(ch)
    # warmup (not timed): one short and one long request
    for n in (a.prompt_len, a.long_len):
        stub.Generate(GenerateRequest(prompt="w" * n, max_new_tokens=4, is_greedy=True), timeout=600)

    def one(i, prompt, t_arr):
        times = []
        for tok in stub.GenerateStream(GenerateRequest(prompt=prompt, max_new_tokens=a.gen_len, temperature=1.0,
                                                       top_p=0.95, top_k=50, request_id=f"o{i}"), timeout=1200):
            if tok.finished:
                break
            times.append(time.perf_counter())
        res[i] = (t_arr, times, len(prompt))

    t0 = time.perf_counter()
    threads = []
    for i, (ta, prompt) in enumerate(plan):
        dt = t0 + ta - time.perf_counter()
        if dt > 0:
            time.sleep(dt)
        th = threading.Thread(target=one, args=(i, prompt, time.perf_counter()))
        th.start()
        threads.append(th)
    for th in threads:
        th.join()
    el = time.perf_counter() - t0
    ch.close()
    ttft = [r[1][0] - r[0] for r in res if r[1]]
    tpot = [(r[1][-1] - r[1][0]) / (len(r[1]) - 1) for r in res if len(r[1]) > 1]
    gap = [max(b - c for b, c in zip(r[1][1:], r[1][:-1])) for r in res if len(r[1]) > 1]
    toks = sum(len(r[1]) for r in res)

    def pct(v, q):
        return round(float(np.percentile(v, q)) * 1e3, 2) if v else None

    print(json.dumps({"metric": "serving_open_loop", "value": round(toks / el, 2), "unit": "tokens/s",
                      "rate_rps": a.rate, "requests": len(res), "prompt_len": a.prompt_len, "long_len": a.long_len,
                      "long_frac": a.long_frac, "gen_len": a.gen_len,
                      "p50_ttft_ms": pct(ttft, 50), "p99_ttft_ms": pct(ttft, 99),
                      "p50_tpot_ms": pct(tpot, 50), "p99_tpot_ms": pct(tpot, 99),
                      "p50_max_token_gap_ms": pct(gap, 50), "p99_max_token_gap_ms": pct(gap, 99),
                      "wall_s": round(el, 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--mode", choices=["grpc", "pubsub"], default="grpc")
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=4, help="timed requests per client")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--rate", type=float, default=0.0, help="open loop: Poisson arrivals at this many requests/s")
    ap.add_argument("--num-requests", type=int, default=256, help="open loop: requests in total")
    ap.add_argument("--long-len", type=int, default=2048, help="open loop: length of the long prompts")
    ap.add_argument("--long-frac", type=float, default=0.1, help="open loop: share of long prompts")
    ap.add_argument("--frontend-inproc", action="store_true",
                    help="pubsub: run the broker and the gRPC front-end inside the engine process")
    ap.add_argument("--client-port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--frontend", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--broker", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.broker:  # pub/sub broker role (the Redis server): runs until stdin closes
        from llmss_amd.serving.broker import MiniRedisServer

        mini = MiniRedisServer().start()
        print(mini.port, flush=True)
        sys.stdin.read()
        mini.stop()
        return
    if a.frontend:  # pub/sub front-end role: gRPC front-end on a broker in its own process; runs until stdin closes
        from llmss_amd.serving.grpc_api import AioBrokerServicer, serve

        br = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--broker"], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
        port = int(br.stdout.readline())
        srv = serve(AioBrokerServicer("127.0.0.1", port), port=0, host="127.0.0.1")
        print(f"{port} {srv.bound_port}", flush=True)
        sys.stdin.read()
        srv.stop(0).wait(30)
        br.stdin.close()
        br.wait(30)
        return

    if a.client_port:
        if a.client_port < 0:  # spawned before the parent touched the GPU; the port comes on stdin
            a.client_port = int(sys.stdin.readline())
        return run_open_loop(a) if a.rate > 0 else run_clients(a)

    # the clients run in their own process (no GPU, no shared GIL with the engine loop); it is started
    # before this process initialises the GPU and learns the server port on stdin
    cmd = [sys.executable, os.path.abspath(__file__), "--client-port=-1"] + [
        f"--{k.replace('_', '-')}={v}" for k, v in vars(a).items()
        if k in ("clients", "requests", "prompt_len", "gen_len", "rate", "num_requests", "long_len", "long_frac")]
    child = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    fe = None
    if a.mode == "pubsub" and not a.frontend_inproc:  # started before this process touches the GPU
        fe = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--frontend"], stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
        fe_broker_port, fe_grpc_port = map(int, fe.stdout.readline().split())

    import torch

    from llmss_amd.engine import LLMEngine, build_model
    from llmss_amd.serving.broker import MiniRedisServer, RedisBroker
    from llmss_amd.serving.consumer import Consumer
    from llmss_amd.serving.driver import EngineDriver
    from llmss_amd.serving.grpc_api import AioBrokerServicer, EngineServicer, serve
    from llmss_amd.utils.tokenizer import load_tokenizer

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = build_model(a.model, None, "bf16" if dev.type == "cuda" else "fp32", dev, fp8=a.fp8, random_init=True)
    tok = load_tokenizer(a.model, model.cfg.vocab_size)
    longest = max(a.prompt_len, a.long_len if a.rate > 0 else 0)
    eng = LLMEngine(model, max_num_seqs=a.clients, max_batched_tokens=max(8192, a.clients * a.prompt_len),
                    max_model_len=min(model.cfg.max_position_embeddings, longest + a.gen_len + 8))
    drv = EngineDriver(eng).start()
    servers, consumer, mini = [], None, None
    if a.mode == "grpc":
        srv = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
        servers.append(srv)
        port = srv.bound_port
    elif fe is not None:
        consumer = Consumer(drv, tok, RedisBroker("127.0.0.1", fe_broker_port), poll_timeout=0.05).start()
        port = fe_grpc_port
    else:
        mini = MiniRedisServer().start()
        consumer = Consumer(drv, tok, RedisBroker(mini.host, mini.port), poll_timeout=0.05).start()
        srv = serve(AioBrokerServicer(mini.host, mini.port), port=0, host="127.0.0.1")
        servers.append(srv)
        port = srv.bound_port
    out, _ = child.communicate(f"{port}\n", timeout=1800)
    if child.returncode:
        raise RuntimeError(f"client process failed with exit code {child.returncode}")
    res = json.loads(out.strip().splitlines()[-1])
    res.update(mode=a.mode, model=a.model, fp8=a.fp8, data="synthetic prompts, random-init weights",
               frontend=None if a.mode == "grpc" else ("in-process" if fe is None else "own process"),
               prefill_chunk=eng.prefill_chunk, engine_stats=eng.stats,
               driver_stats={k: v for k, v in drv.stats.items() if k.startswith("admit")},
               admissions=list(drv.admit_log)[-48:])
    print(json.dumps(res), flush=True)
    # orderly shutdown: front-ends first, then the engine thread, then device state. A teardown that takes
    # over a minute dumps every thread's stack (a run once went silent here after printing its result)
    faulthandler.dump_traceback_later(60, exit=False)
    for s in servers:
        s.stop(0).wait(60)
    if consumer is not None:
        consumer.stop()
    if mini is not None:
        mini.stop()
    if fe is not None:
        fe.stdin.close()
        fe.wait(60)
    drv.stop()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
