"""Decode-graph capture is agreed across TP ranks: when capture fails on ONE rank, every rank
drops its graphs and decodes eagerly, the post-capture consistency check passes, and generation still matches
across ranks - no rank is left waiting in a collective (the capture-time A/B's all_gather_object) that a peer
never joins. CPU / gloo: the capture itself is stubbed (a no-op that succeeds), the failure is injected on rank 1
with LLMSS_FAULT_INJECT="1:capture:raise"."""
import os
import socket

import torch
import torch.multiprocessing as mp

from helpers import save_hf_model


def _worker(rank, port, ckpt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank), LLMSS_FAULT_INJECT="1:capture:raise")
    torch.set_num_threads(1)
    try:
        from llmss_amd.engine import LLMEngine, SamplingParams, build_model
        from llmss_amd.parallel.dist import initialize_distributed

        tp, r, _ = initialize_distributed(backend="gloo")
        ok, err = tp.agree(lambda: (_ for _ in ()).throw(RuntimeError("boom")) if r == 0 else None)
        assert (ok, err) == (False, "RuntimeError: boom" if r == 0 else ""), (ok, err)
        assert tp.agree(lambda: None) == (True, "")
        # any exception type is agreed (a ValueError / HIP error on one rank must not make it leave alone)
        ok, err = tp.agree(lambda: int("x") if r == 1 else None)
        assert not ok and (err.startswith("ValueError") if r == 1 else err == ""), (ok, err)
        m = build_model(ckpt, tp, "fp32", "cpu")
        eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64, check_tokens=True)
        calls = []
        eng.capture_graphs = lambda: calls.append(1)  # the GPU capture, stubbed: succeeds wherever it runs
        eng.use_graphs = True
        eng._capture_agreed()
        assert not eng.use_graphs and not eng.graphs
        assert calls == ([1] if r == 0 else [])  # rank 1 failed before capturing
        out = eng.generate([[1, 2, 3, 4], [5, 6, 7]], SamplingParams(max_new_tokens=5, is_greedy=True,
                                                                      ignore_eos=True))
        q.put((r, out))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_capture_failure_on_one_rank_is_agreed(tmp_path):
    d = str(tmp_path / "llama")
    save_hf_model("llama", d, vocab=101)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(i, port, d, q)) for i in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=180) for _ in range(2))
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert isinstance(got[0], list) and got[0] == got[1], got
    assert [p.exitcode for p in procs] == [0, 0]


def _preinit_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        import torch.distributed as dist

        from llmss_amd.parallel import dist as D

        dist.init_process_group("gloo", rank=rank, world_size=2)
        fail = rank == 1
        real = torch.cuda.set_device
        if fail:  # rank 1's device step fails; rank 0's succeeds (stubbed: no GPU here)
            torch.cuda.set_device = lambda *a: (_ for _ in ()).throw(RuntimeError("no device"))
        else:
            torch.cuda.set_device = lambda *a: None
            torch.cuda.synchronize = lambda *a: None
        torch.cuda.current_device = lambda: 0
        try:
            D._native_comm(rank, 1, 2)
            q.put((rank, "returned"))
        except RuntimeError as e:
            q.put((rank, str(e)))
        finally:
            torch.cuda.set_device = real
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "unexpected " + repr(e)))


def test_rccl_preinit_failure_on_one_rank_raises_on_all():
    """parallel/dist.py _native_comm: a rank whose pre-init step fails (here its device) makes EVERY rank raise
    before ncclCommInitRank, instead of leaving the healthy rank blocked in the init."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_preinit_worker, args=(i, port, q)) for i in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=120) for _ in range(2))
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert "pre-init check failed (device: no device)" in got[1], got
    assert "pre-init check failed (on a peer)" in got[0], got
