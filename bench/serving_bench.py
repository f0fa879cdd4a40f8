"""Serving benchmark: concurrent gRPC clients against the engine (BASELINE: "GPT-2-XL TP=1 bf16 on
one MI355X served over gRPC"; "pubsub producer/consumer under concurrent gRPC clients").

  --mode grpc    clients -> gRPC Generate service on the engine driver (direct)
  --mode pubsub  clients -> gRPC front-end -> RESP broker (mini Redis) -> consumer -> engine

Random-init weights of the named architecture, random printable prompts (byte tokenizer: one
token per character). Prints one JSON line: output tokens/s over the timed requests, p50 request
latency and p50 server-side TTFT.

usage: python bench/serving_bench.py [--model gpt2-xl] [--mode grpc|pubsub] [--clients 64] [--requests 4]
"""
import argparse
import concurrent.futures as cf
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--mode", choices=["grpc", "pubsub"], default="grpc")
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=4, help="timed requests per client")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--client-port", type=int, default=0, help=argparse.SUPPRESS)
    a = ap.parse_args()

    if a.client_port:
        if a.client_port < 0:  # spawned before the parent touched the GPU; the port comes on stdin
            a.client_port = int(sys.stdin.readline())
        return run_clients(a)

    # the clients run in their own process (no GPU, no shared GIL with the engine loop); it is started
    # before this process initialises the GPU and learns the server port on stdin
    cmd = [sys.executable, os.path.abspath(__file__), "--client-port=-1"] + [
        f"--{k.replace('_', '-')}={v}" for k, v in vars(a).items() if k in ("clients", "requests", "prompt_len", "gen_len")]
    child = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)

    import torch

    from llmss_amd.engine import LLMEngine, build_model
    from llmss_amd.serving.broker import MiniRedisServer, RedisBroker
    from llmss_amd.serving.consumer import Consumer
    from llmss_amd.serving.driver import EngineDriver
    from llmss_amd.serving.grpc_api import BrokerServicer, EngineServicer, serve
    from llmss_amd.utils.tokenizer import load_tokenizer

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = build_model(a.model, None, "bf16" if dev.type == "cuda" else "fp32", dev, fp8=a.fp8, random_init=True)
    tok = load_tokenizer(a.model, model.cfg.vocab_size)
    eng = LLMEngine(model, max_num_seqs=a.clients, max_batched_tokens=max(8192, a.clients * a.prompt_len),
                    max_model_len=min(model.cfg.max_position_embeddings, a.prompt_len + a.gen_len + 8))
    drv = EngineDriver(eng).start()
    servers, consumer, mini = [], None, None
    if a.mode == "grpc":
        srv = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
    else:
        mini = MiniRedisServer().start()
        consumer = Consumer(drv, tok, RedisBroker(mini.host, mini.port), poll_timeout=0.05).start()
        srv = serve(BrokerServicer(RedisBroker(mini.host, mini.port)), port=0, host="127.0.0.1")
    servers.append(srv)
    out, _ = child.communicate(f"{srv.bound_port}\n", timeout=1800)
    if child.returncode:
        raise RuntimeError(f"client process failed with exit code {child.returncode}")
    res = json.loads(out.strip().splitlines()[-1])
    res.update(mode=a.mode, model=a.model, fp8=a.fp8, data="synthetic prompts, random-init weights")
    print(json.dumps(res), flush=True)
    # orderly shutdown: front-ends first, then the engine thread, then device state
    for s in servers:
        s.stop(0).wait()
    if consumer is not None:
        consumer.stop()
    if mini is not None:
        mini.stop()
    drv.stop()
    if dev.type == "cuda":
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
