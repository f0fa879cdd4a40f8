"""Functional rehearsal of the driver's multi-GPU bench invocation on the CPU: two ranks launched as
torchrun would (RANK / WORLD_SIZE / MASTER_* env, 127.0.0.1), gloo instead of RCCL, tiny models. Covers
bench.py's N>1 path end to end: TP=2 engine in lock-step on both ranks, barrier-bracketed timing, MAX of
the per-rank clocks, the data-parallel secondary config (SUM of tokens) and the single rank-0 JSON line."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [2, 8])
def test_bench_two_ranks_gloo(n):
    """n = 8: the driver's full-node invocation rehearsed rank for rank (TP=8 over 8 gloo processes, a 16-head tiny
    Llama: 2 heads per rank)."""
    port = _free_port()
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--model",
            "tiny-llama" if n <= 4 else "tiny-llama16h", "--secondary",
            "tiny-gpt2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2", "--prompt-len", "8", "--gen-len", "4"]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen(args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=ROOT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=420))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not [ln for o, _ in outs[1:] for ln in o.splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 2 and d["config"]["parallelism"] == f"tp{n}"
    assert d["config"]["global_batch"] == 2 * n and len(d["rank_elapsed_s"]) == n
    # TP: every rank generates the same 2n x 4 tokens per step, counted once
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 8 * n) < 0.05 * n  # value and ms_per_step are rounded
    s = d["secondary"]
    assert s["config"]["parallelism"] == f"dp{n}xtp1" and s["config"]["global_batch"] == 2 * n
    assert abs(s["value"] * s["ms_per_step"] / 1e3 - 8 * n) < 0.05 * n  # n replicas x 2 requests x 4 tokens


def _cpu_env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", **kw)
    return env


_TINY = ["--model", "tiny-llama", "--secondary", "none", "--batch-per-gpu", "2", "--prompt-len", "8", "--gen-len", "4"]


def test_bench_self_launches_ranks():
    """`python bench.py --gpus 2` without torchrun: the process becomes a launcher for 2 ranks and forwards
    rank 0's single JSON line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"]
                       + _TINY, env=_cpu_env(), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tp2" and d["rccl_world_size"] == 2
    assert len(d["rank_elapsed_s"]) == 2 and max(d["rank_elapsed_s"]) * 1e3 / 2 == pytest.approx(d["ms_per_step"],
                                                                                                 rel=1e-2)


@pytest.mark.parametrize("kind", ["exit", "raise", "hang"])
def test_bench_launcher_fails_fast_on_rank_failure(kind):
    """One rank dies (or hangs) mid-run: the launcher stops every rank and exits non-zero naming it."""
    timeout = "40" if kind == "hang" else "600"
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--timeout", timeout] + _TINY, env=_cpu_env(LLMSS_FAULT_INJECT=f"1:1:{kind}"),
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if kind == "hang":
        assert r.returncode == 124 and "timeout" in r.stderr
    else:
        assert "rank 1 exited" in r.stderr or "rank 0 exited" in r.stderr, r.stderr[-2000:]
    assert time.time() - t0 < 200
