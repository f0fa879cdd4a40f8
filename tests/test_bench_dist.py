"""Functional rehearsal of the driver's multi-GPU bench invocation on the CPU: two ranks launched as
torchrun would (RANK / WORLD_SIZE / MASTER_* env, 127.0.0.1), gloo instead of RCCL, tiny models. Covers
bench.py's N>1 path end to end: TP=2 engine in lock-step on both ranks, barrier-bracketed timing, MAX of
the per-rank clocks, the data-parallel secondary config (SUM of tokens) and the single rank-0 JSON line."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo():
    port = _free_port()
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny-llama", "--secondary",
            "tiny-gpt2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2", "--prompt-len", "8", "--gen-len", "4"]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen(args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=ROOT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["config"]["parallelism"] == "tp2"
    assert d["config"]["global_batch"] == 4
    # TP: both ranks generate the same 4 x 4 tokens per step, counted once
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 16) < 0.05  # value and ms_per_step are rounded
    s = d["secondary"]
    assert s["config"]["parallelism"] == "dp2xtp1" and s["config"]["global_batch"] == 4
    assert abs(s["value"] * s["ms_per_step"] / 1e3 - 16) < 0.05  # 2 replicas x 2 requests x 4 tokens
