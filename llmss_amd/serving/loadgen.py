"""Closed-batch gRPC load generator (client process of ``bench.py``'s served configuration).

BASELINE config #2 is "GPT-2-XL TP=1 bf16 on one MI355X served over gRPC" - the reference serves its
model over HTTP -> Redis -> consumer (``poc-server/producer-consumer/producer_server.py:45-55``) and has
no gRPC. ``bench.py`` runs the engine behind the in-process gRPC ``Generate`` service and this process
acts as the clients: it is started before the bench touches the GPU, learns the server port on stdin,
then executes one *step* per ``step`` line - ``batch`` concurrent ``Generate`` calls with synthetic
pre-tokenized prompts (``prompt_token_ids``) - and answers with one JSON line (tokens received, per-request
latency / server TTFT / TPOT). ``quit`` ends it. ``bench.py`` runs several of these processes side by side
(``--clients``), each with its share of the step's requests, as independent clients would.

usage: python -m llmss_amd.serving.loadgen --batch 64 --prompt-len 128 --gen-len 128 --vocab 50257
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import numpy as np


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--prompt-len", type=int, required=True)
    ap.add_argument("--gen-len", type=int, required=True)
    ap.add_argument("--vocab", type=int, required=True)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--greedy", action="store_true")
    a = ap.parse_args(argv)

    import grpc

    from .grpc_api import GenerateRequest, Stub

    line = sys.stdin.readline()
    if not line:
        return 0
    port = int(line)
    ch = grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_receive_message_length", 64 << 20)])
    grpc.channel_ready_future(ch).result(timeout=120)
    stub = Stub(ch)
    rng = np.random.default_rng(a.seed)
    step = 0
    for cmd in sys.stdin:
        cmd = cmd.strip()
        if cmd == "quit":
            break
        if cmd != "step":
            continue
        reqs = [GenerateRequest(prompt_token_ids=rng.integers(0, a.vocab, a.prompt_len).tolist(),
                                max_new_tokens=a.gen_len, is_greedy=a.greedy, temperature=1.0, top_p=0.95, top_k=50,
                                seed=7 + i, ignore_eos=True, request_id=f"s{step}r{i}") for i in range(a.batch)]
        t0 = time.perf_counter()
        futs = [(time.perf_counter(), stub.Generate.future(r, timeout=1800)) for r in reqs]
        lat, ttft, tpot, ntok = [], [], [], 0
        for ts, f in futs:
            resp = f.result()
            n = len(resp.token_ids)
            ntok += n
            lat.append(time.perf_counter() - ts)
            ttft.append(float(resp.ttft_s))
            if n > 1:
                tpot.append((float(resp.e2e_s) - float(resp.ttft_s)) / (n - 1))
        print(json.dumps({"step": step, "tokens": ntok, "wall_s": time.perf_counter() - t0,
                          "p50_latency_s": float(np.median(lat)), "p50_ttft_s": float(np.median(ttft)),
                          "p50_tpot_s": float(np.median(tpot)) if tpot else None,
                          "latency_s": lat, "ttft_s": ttft, "tpot_s": tpot}), flush=True)
        step += 1
    ch.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
