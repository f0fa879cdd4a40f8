"""Headline benchmark: output tokens/s (node) + p50 latency for batched generation.

Config (BASELINE.json): Llama-2-7B with tensor parallelism TP = N (one process per GPU, RCCL over
xGMI; TP=8 at N=8) - or ``--model gpt2-xl`` for the GPT-2-XL TP=1 configuration. Random-init
weights of the exact architecture and synthetic prompt token ids (no network, no checkpoints).

A "step" = one complete batched generation through the serving engine: ``batch`` synthetic
prompts of ``--prompt-len`` tokens, prefill + ``--gen-len`` decode tokens each (continuous-
batching scheduler, paged KV cache, HIP-graph decode, on-device sampling with the reference's
default temperature=1.0 / top_p=0.95 / top_k=50). Weak scaling: the global batch is
``--batch-per-gpu * N``. ``value`` = total generated tokens / wall time over all ranks (max).

Launch: ``python bench.py`` (N=1), ``python bench.py --gpus N`` (this process becomes a GPU-free
launcher: it starts N rank processes of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
forwards rank 0's JSON line, and on any rank failure or the ``--timeout`` kills the others and exits
non-zero naming the rank), or ``torchrun --nproc-per-node N bench.py --gpus N`` (each rank directly).
Reference launch recipe: ``torchrun --nproc_per_node 4 consumer_server.py``
(``poc-server/producer-consumer/README.md:29-36``), ``initialize_torch_distributed`` (``dist.py:40-77``).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"],
                    help="paged KV cache storage: bf16, or fp8 e4m3 rows with per-row scales")
    ap.add_argument("--greedy", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--secondary", default="gpt2-xl",
                    help="second headline model timed after the first (TP=1 per GPU, data-parallel over N GPUs); "
                         "'' or 'none' to skip")
    ap.add_argument("--simulate-tp", type=int, default=0,
                    help="dev tool: one process computes rank 0 of a TP=N shard plan with no communication "
                         "(per-rank compute time at TP=N shapes; not a headline number)")
    ap.add_argument("--sim-comm", default="",
                    help="with --simulate-tp: model each all-reduce / all-gather as LAT_US,GBPS[,CHANNELS] (latency + "
                         "bytes / algorithmic bandwidth on the collective's stream: a one-workgroup spin kernel, or "
                         "CHANNELS workgroups moving the collective's memory traffic) to measure comm overlap")
    ap.add_argument("--sim-tbo", type=int, default=0,
                    help="with --simulate-tp and --sim-comm: run decode steps of >= N sequences as two micro-batches "
                         "(the overlap schedule the real communicator's capture-time A/B can pick)")
    ap.add_argument("--clients", type=int, default=4,
                    help="gRPC client processes for the served secondary config (each sends its share of the "
                         "step's concurrent requests)")
    ap.add_argument("--secondary-serve", default="grpc", choices=["grpc", "engine"],
                    help="secondary config timed through the in-process gRPC Generate service with a separate "
                         "client process (BASELINE config #2 'served over gRPC'; the engine-direct number is "
                         "reported too), or engine-direct only")
    ap.add_argument("--timeout", type=float, default=float(os.environ.get("LLMSS_BENCH_TIMEOUT_S", "2400")),
                    help="launcher mode: kill every rank and exit 124 after this many seconds")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))

    # the gRPC clients run in their own process, started before this one touches the GPU (no fork of a
    # GPU-initialised process); they learn the server port on stdin once the engine is up
    client = None
    if args.secondary not in ("", "none") and args.secondary != args.model and args.simulate_tp <= 1 \
            and args.secondary_serve == "grpc":
        from llmss_amd.models.config import get_preset

        nc = max(1, min(args.clients, args.batch_per_gpu))
        share = [args.batch_per_gpu // nc + (i < args.batch_per_gpu % nc) for i in range(nc)]
        client = [subprocess.Popen(
            [sys.executable, "-m", "llmss_amd.serving.loadgen", "--batch", str(share[i]), "--prompt-len",
             str(args.prompt_len), "--gen-len", str(args.gen_len), "--vocab", str(get_preset(args.secondary).vocab_size),
             "--seed", str(4321 + 97 * i + int(os.environ.get("RANK", "0")))] + (["--greedy"] if args.greedy else []),
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=ROOT) for i in range(nc)]

    from llmss_amd.models.config import get_preset
    from llmss_amd.parallel.dist import RCCL_TUNE_INFO, TPGroup, initialize_distributed

    if args.gpus > 1:  # the start-up RCCL setting probe times the decode all-reduce of THIS run: rows x hidden bf16
        os.environ.setdefault("LLMSS_RCCL_TUNE_BYTES", str(args.batch_per_gpu * args.gpus *
                                                           get_preset(args.model).hidden_size * 2))
    tp, rank, world = initialize_distributed()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.simulate_tp > 1:
        if world != 1:
            raise SystemExit("--simulate-tp runs in a single process")
        sim = tuple(float(v) for v in args.sim_comm.split(",")) if args.sim_comm else None
        tp = TPGroup(0, args.simulate_tp, fake=True, sim_comm=sim)
        tp.replicate_gather = True  # the gathered candidates / logits have their TP=N width

    def progress(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    if world > 1 and args.simulate_tp <= 1 and torch.cuda.is_available() and tp.comm is not None:
        comm = comm_probe(tp, progress)
    else:
        comm = None
    res = run_config(args, args.model, tp, args.batch_per_gpu * max(world, args.simulate_tp), progress)
    if comm is not None:
        res["comm_probe"] = comm
    if RCCL_TUNE_INFO:
        res["rccl_setting_probe"] = dict(RCCL_TUNE_INFO)
    if args.secondary not in ("", "none") and args.simulate_tp <= 1 and args.secondary != args.model:
        # second BASELINE headline config (GPT-2-XL TP=1, 25 heads: no TP split), driver-timed in the same run;
        # with N GPUs every rank serves its own TP=1 replica (data parallel) and the node total is reported
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        res["secondary"] = run_config(args, args.secondary, tp, args.batch_per_gpu * world, progress, dp=True,
                                      client=client)
    for c in client or []:
        if c.poll() is None:
            c.stdin.write("quit\n")
            c.stdin.flush()
            c.wait(timeout=60)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if tp.is_real:
        tp.close()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


# ------------------------------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pump(stream, sink, keep):
    """Copy a child's stream line by line into `sink` (None: drop) and keep the last lines in `keep`."""
    for line in iter(stream.readline, ""):
        keep.append(line)
        if sink is not None:
            sink.write(line)
            sink.flush()
    stream.close()


def launch(args) -> int:
    """GPU-free parent: start ``args.gpus`` rank processes of this script (no exec, no GPU call here),
    forward rank 0's stdout (the JSON line) and stderr (progress), and fail fast: the first rank that
    exits non-zero, or the timeout, ends every rank; the exit code is the failing rank's (124 on
    timeout) and stderr names the rank with the tail of its stderr."""
    n = args.gpus
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    argv = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    procs, tails, pumps = [], [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        p = subprocess.Popen(argv, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        out_tail, err_tail = collections.deque(maxlen=400), collections.deque(maxlen=60)
        for stream, sink, keep in ((p.stdout, sys.stdout if r == 0 else None, out_tail),
                                   (p.stderr, sys.stderr if r == 0 else None, err_tail)):
            th = threading.Thread(target=_pump, args=(stream, sink, keep), daemon=True)
            th.start()
            pumps.append(th)
        procs.append(p)
        tails.append(err_tail)

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def fail(r, code, why):
        kill_all()
        for th in pumps:
            th.join(timeout=2)
        tail = "".join(tails[r]) if r is not None else ""
        print(f"[bench launcher] {why}; stopped all {n} ranks\n--- rank {r} stderr (tail) ---\n{tail}",
              file=sys.stderr, flush=True)
        return code

    t0 = time.time()
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                return fail(r, c if c > 0 else 128 - c, f"rank {r} exited with code {c}")
            if all(c == 0 for c in codes):
                break
            if time.time() - t0 > args.timeout:
                r = next((i for i, c in enumerate(codes) if c is None), None)
                return fail(r, 124, f"timeout after {args.timeout:.0f}s (rank {r} still running)")
            time.sleep(0.2)
    except KeyboardInterrupt:
        return fail(None, 130, "interrupted")
    for th in pumps:
        th.join(timeout=10)
    return 0


# ------------------------------------------------------------------------------------------ comm probe
def comm_probe(tp, progress) -> dict:
    """Latency of the native RCCL all-reduce at decode / prefill message sizes, eager and inside a HIP
    graph (20 back-to-back all-reduces per replay): per-collective microseconds on this node's xGMI."""
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {}
    for nbytes in (64 << 10, 512 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
        x = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=dev)
        for _ in range(3):
            tp.all_reduce(x)
        torch.cuda.synchronize()
        tp.barrier()
        n = 20
        t = time.perf_counter()
        for _ in range(n):
            tp.all_reduce(x)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t) / n * 1e6
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            tp.all_reduce(x)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(n):
                tp.all_reduce(x)
        g.replay()
        torch.cuda.synchronize()
        tp.barrier()
        t = time.perf_counter()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t) / (3 * n) * 1e6
        out[str(nbytes)] = {"eager_us": round(eager, 1), "graph_us": round(graph, 1),
                            "busbw_GBps": round(2 * (tp.size - 1) / tp.size * nbytes / graph / 1e3, 1)}
        del g, x
    progress(f"comm probe ({tp.backend}, {tp.size} ranks): " +
             ", ".join(f"{int(k) >> 10}KiB {v['graph_us']}us" for k, v in out.items()))
    return {"backend": tp.backend, "ranks": tp.size, "all_reduce_bf16": out}


def runtime_record(tp, eng, dp: bool) -> dict:
    """What this rank's number depends on besides the code: data plane, RCCL library version, every NCCL_* /
    RCCL_* / HSA_* variable in the environment, whether decode ran in HIP graphs (and which buckets), and the
    capture-time micro-batch A/B's choice."""
    rec = {"rank": tp.global_rank if tp.is_real else int(os.environ.get("RANK", "0")),
           "data_plane": "none (independent replicas)" if dp else tp.backend,
           "device": torch.cuda.get_device_name() if torch.cuda.is_available() else "cpu",
           "use_graphs": bool(eng.use_graphs), "graph_buckets": sorted({b for b, _ in eng.graphs}),
           "decode_schedule": {str(b): v for b, v in sorted(eng.decode_schedule.items())},
           "env": {k: v for k, v in sorted(os.environ.items())
                   if k.startswith(("NCCL_", "RCCL_", "HSA_", "LLMSS_", "TORCH_NCCL_", "GPU_MAX_HW_QUEUES"))}}
    try:
        from llmss_amd import _native

        rec["rccl_version"] = _native().rccl_version()
    except Exception as e:  # noqa: BLE001 - CPU rehearsal without the extension
        rec["rccl_version"] = f"unavailable ({type(e).__name__})"
    return rec


def _world_gather(obj):
    out = [None] * torch.distributed.get_world_size()
    torch.distributed.all_gather_object(out, obj)
    return out


def run_served(args, eng, client, progress, world, rank_sync):
    """The same engine behind the in-process gRPC Generate service (EngineDriver thread + EngineServicer);
    the client processes send each step's ``batch`` requests concurrently. Returns (seconds, tokens, client
    step reports) over ``args.steps`` timed steps after ``args.warmup`` untimed ones."""
    from llmss_amd.serving.driver import EngineDriver
    from llmss_amd.serving.grpc_api import EngineServicer, serve
    from llmss_amd.utils.tokenizer import load_tokenizer

    drv = EngineDriver(eng).start()
    server = serve(EngineServicer(drv, load_tokenizer(args.secondary, eng.cfg.vocab_size)), port=0, host="127.0.0.1")
    for c in client:
        c.stdin.write(f"{server.bound_port}\n")
        c.stdin.flush()

    def step():
        for c in client:  # every client process sends its share of the step's requests at once
            c.stdin.write("step\n")
            c.stdin.flush()
        reps = []
        for c in client:
            line = c.stdout.readline()
            if not line:
                raise RuntimeError(f"gRPC client process ended (exit code {c.poll()})")
            reps.append(json.loads(line))
        lat = [v for r in reps for v in r["latency_s"]]
        ttft = [v for r in reps for v in r["ttft_s"]]
        tpot = [v for r in reps for v in r["tpot_s"]]
        return {"tokens": sum(r["tokens"] for r in reps), "wall_s": max(r["wall_s"] for r in reps),
                "p50_latency_s": float(np.median(lat)), "p50_ttft_s": float(np.median(ttft)),
                "p50_tpot_s": float(np.median(tpot)) if tpot else None}

    try:
        for i in range(args.warmup):
            r = step()
            progress(f"grpc warmup {i}: {r['wall_s']:.3f}s")
        rank_sync()
        t0 = time.perf_counter()
        reps = []
        for i in range(args.steps):
            reps.append(step())
            progress(f"grpc step {i}: {reps[-1]['tokens']} tokens, {time.perf_counter() - t0:.3f}s elapsed")
        rank_sync()
        el = time.perf_counter() - t0
        dstats = dict(drv.stats, ctrl=drv.ctrl)
    finally:
        server.stop(0).wait()
        drv.stop()
    if drv.error is not None:
        raise RuntimeError(f"engine driver failed: {drv.error}")
    reps[0]["driver_stats"] = dstats
    return el, sum(r["tokens"] for r in reps), reps


def run_config(args, model_name, tp, batch, progress, dp=False, client=None):
    """Build ``model_name`` on ``tp`` (``dp``: an independent TP=1 replica per rank), warm up, time
    ``args.steps`` batched generations; returns the JSON dict."""
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    world = args.gpus
    # GPU: this rank's device. CPU (no GPU): the PyTorch reference path over gloo - a functional rehearsal
    # of the multi-rank bench (tests/test_bench_dist.py), not a performance number
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    local_batch = batch // world if dp else batch
    t_setup = time.perf_counter()
    model = build_model(model_name, tp if not dp else None, "bf16", dev, fp8=args.fp8, random_init=True)
    if args.simulate_tp > 1 and args.sim_tbo:  # dev tool: decode steps of >= N sequences as two micro-batches
        model.tbo_min = args.sim_tbo
    t_model = time.perf_counter() - t_setup
    max_len = min(model.cfg.max_position_embeddings, max(256, args.prompt_len + args.gen_len))
    eng = LLMEngine(model, max_num_seqs=local_batch, max_batched_tokens=max(8192, local_batch * args.prompt_len),
                    block_size=16, max_model_len=max_len, use_graphs=not args.no_graphs, kv_dtype=args.kv_dtype)
    # engine init = KV pool + GEMM autotune + attention routing + decode-graph capture (and its TBO A/B)
    setup_s = {"model": round(t_model, 2), "engine": round(time.perf_counter() - t_setup - t_model, 2)}
    rng = np.random.default_rng(1234 + (tp.rank if dp else 0))
    V = model.cfg.vocab_size

    def prompts():
        return [rng.integers(0, V, args.prompt_len).tolist() for _ in range(local_batch)]

    def params():
        return SamplingParams(max_new_tokens=args.gen_len, is_greedy=args.greedy, temperature=1.0, top_p=0.95,
                              top_k=50, ignore_eos=True, seed=7)

    fault = os.environ.get("LLMSS_FAULT_INJECT", "")  # "rank:step:kind" (kind exit | raise | hang), tests only
    fault = tuple(fault.split(":")) if fault else None
    my_rank = tp.global_rank if tp.is_real else int(os.environ.get("RANK", "0"))
    steps_done = [0]

    def one_step():
        if fault is not None and int(fault[0]) == my_rank and int(fault[1]) == steps_done[0]:
            progress(f"rank {my_rank}: injected fault {fault[2]!r} at step {steps_done[0]}")
            if fault[2] == "exit":
                os._exit(17)
            if fault[2] == "hang":
                time.sleep(1e6)
            raise RuntimeError(f"injected fault at bench step {steps_done[0]}")
        steps_done[0] += 1
        for p in prompts():
            eng.add_request(p, params())
        n = 0
        while eng.has_unfinished():
            n += len(eng.step())
        reqs = eng.pop_finished()
        return n, [r.metrics() for r in reqs]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def barrier():
        if world > 1 and args.simulate_tp <= 1:
            torch.distributed.barrier()  # CPU (gloo) group with the native RCCL data plane

    progress(f"engine ready: {model.cfg.model_type} {'dp' if dp else 'tp'}={world} batch={batch} "
             f"kv_blocks={eng.num_blocks} graphs={sorted({b for b, _ in eng.graphs})} setup_s={setup_s}")
    if eng.tuned:
        mx = max(m for _, m in eng.tuned)
        progress("autotuned GEMMs at M=%d: " % mx + ", ".join(
            f"{n} {nt:#x}/s{sp} {t:.1f}us (static {t0:.1f})" for (n, m), (nt, sp, t, t0) in sorted(eng.tuned.items())
            if m == mx))
    for i in range(args.warmup):
        t = time.perf_counter()
        one_step()
        progress(f"warmup {i}: {time.perf_counter() - t:.3f}s")
    barrier()
    sync()
    t0 = time.perf_counter()
    total, mets = 0, []
    for i in range(args.steps):
        n, m = one_step()
        total += n
        mets.extend(m)
        progress(f"step {i}: {n} tokens, {time.perf_counter() - t0:.3f}s elapsed")
    sync()
    barrier()
    el = time.perf_counter() - t0
    rank_el = [el]
    rt = [runtime_record(tp, eng, dp)]
    if world > 1 and args.simulate_tp <= 1:
        rt = tp.all_gather_object(rt[0]) if not dp else _world_gather(rt[0])
    if world > 1 and args.simulate_tp <= 1:  # slowest rank's clock; node total of generated tokens
        allv = tp.all_gather_object((el, total)) if not dp else _world_gather((el, total))
        rank_el = [v[0] for v in allv]
        el = max(rank_el)
        total = sum(v[1] for v in allv) if dp else allv[0][1]
    tpot = np.nanmedian([m["tpot_s"] for m in mets]) * 1e3
    ttft = np.nanmedian([m["ttft_s"] for m in mets]) * 1e3
    e2e = np.nanmedian([m["e2e_s"] for m in mets]) * 1e3
    value = total / el
    if args.simulate_tp > 1:
        par = f"tp{args.simulate_tp}-simulated-" + (f"comm-model-{args.sim_comm}" if args.sim_comm else "no-comm") + (
            f"-tbo{args.sim_tbo}" if args.sim_tbo else "")
    else:
        par = (f"dp{world}xtp1" if world > 1 else "tp1") if dp else f"tp{world}"
    out = {
        "metric": "output_tokens_per_sec",
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8-weights/bf16" if args.fp8 else "bf16",
        "data": "synthetic prompts, random-init weights",
        "rccl_world_size": (torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1),
        "comm_backend": tp.backend if not dp else "none (independent replicas)",
        "rank_elapsed_s": [round(v, 4) for v in rank_el],
        "setup_s": setup_s,
        "runtime": rt,
        "p50_tpot_ms": round(float(tpot), 3),
        "p50_ttft_ms": round(float(ttft), 3),
        "p50_request_latency_ms": round(float(e2e), 3),
        "config": {"model": model_name, "global_batch": batch, "seq_len": args.prompt_len + args.gen_len,
                   "prompt_len": args.prompt_len, "gen_len": args.gen_len, "parallelism": par,
                   "sampling": "greedy" if args.greedy else "temperature=1.0,top_p=0.95,top_k=50",
                   "kv_cache": args.kv_dtype,
                   "engine_stats": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()},
                   **({"phase_ms": eng.phase_summary()} if eng.timer.enabled else {})},
    }
    if client is not None:
        def rank_sync():
            sync()
            barrier()
            sync()

        gel, gtot, reps = run_served(args, eng, client, progress, world, rank_sync)
        grank = [gel]
        if world > 1:
            allv = _world_gather((gel, gtot))
            grank = [v[0] for v in allv]
            gel, gtot = max(grank), sum(v[1] for v in allv)
        engine_direct = {k: out[k] for k in ("value", "ms_per_step", "p50_tpot_ms", "p50_ttft_ms",
                                             "p50_request_latency_ms", "rank_elapsed_s")}
        out.update(value=round(gtot / gel, 2), ms_per_step=round(gel / args.steps * 1e3, 3),
                   p50_tpot_ms=round(float(np.median([r["p50_tpot_s"] for r in reps])) * 1e3, 3),
                   p50_ttft_ms=round(float(np.median([r["p50_ttft_s"] for r in reps])) * 1e3, 3),
                   p50_request_latency_ms=round(float(np.median([r["p50_latency_s"] for r in reps])) * 1e3, 3),
                   rank_elapsed_s=[round(v, 4) for v in grank], engine_direct=engine_direct)
        out["config"]["serving"] = (f"gRPC Generate (in-process grpc.aio server, {local_batch} concurrent requests "
                                    f"per step from {len(client)} client processes); engine_direct = the same "
                                    f"engine stepped directly")
        out["served_over_engine"] = round(out["value"] / engine_direct["value"], 4)
        out["config"]["driver_stats"] = {k: (round(v, 4) if isinstance(v, float) else v)
                                         for k, v in reps[0].get("driver_stats", {}).items()}
        progress(f"served over gRPC: {out['value']} tok/s = {out['served_over_engine']:.1%} of engine-direct "
                 f"{engine_direct['value']}")
    del eng, model
    return out


if __name__ == "__main__":
    main()
