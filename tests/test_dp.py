"""Data-parallel replicas (optional): an in-process Router over independent engines
(least-loaded dispatch, request ids unique across replicas, results identical to one engine) and a
torchrun-style world split into dp x tp groups (dp=2 x tp=2 over gloo: each replica's sharded engine
reproduces TP=1)."""
import os
import socket
import threading

import torch
import torch.multiprocessing as mp

from helpers import save_hf_model


def _prompts(n):
    return [[(7 * i + 3 * j) % 100 for j in range(4 + (i % 5))] for i in range(n)]


def test_router_spreads_and_matches_single_engine(tmp_path):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.serving.driver import EngineDriver
    from llmss_amd.serving.router import Router

    d = str(tmp_path / "llama")
    save_hf_model("llama", d, vocab=101)
    sp = SamplingParams(max_new_tokens=6, is_greedy=True, ignore_eos=True)
    ref = LLMEngine(build_model(d, None, "fp32", "cpu"), max_num_seqs=8, block_size=4, num_blocks=128)
    ps = _prompts(10)
    want = ref.generate(ps, sp)
    reps = [EngineDriver(LLMEngine(build_model(d, None, "fp32", "cpu"), max_num_seqs=4, block_size=4, num_blocks=128))
            for _ in range(2)]
    router = Router(reps).start()
    try:
        hs = [None] * len(ps)

        def go(i):
            hs[i] = router.submit(ps[i], sp)

        th = [threading.Thread(target=go, args=(i,)) for i in range(len(ps))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for h in hs:
            assert h.wait(120)
        assert [h.output_ids for h in hs] == want
        assert len({h.rid for h in hs}) == len(ps)  # ids unique across replicas
        assert all(n > 0 for n in router.routed) and sum(router.routed) == len(ps)
        st = router.engine.stats
        assert st["replicas"] == 2 and all(t > 0 for t in st["per_replica_tokens"])
    finally:
        router.stop()


def _dp_worker(rank, port, d, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="4")
    torch.set_num_threads(1)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed

    tp, r, w = initialize_distributed(backend="gloo", dp=2)
    assert tp.size == 2 and tp.dp == 2 and tp.replica == rank // 2 and tp.rank == rank % 2
    eng = LLMEngine(build_model(d, tp, "fp32", "cpu"), max_num_seqs=4, block_size=4, num_blocks=64, check_tokens=True)
    ps = _prompts(6)[tp.replica::2]  # each replica serves its own requests
    out = eng.generate(ps, SamplingParams(max_new_tokens=6, is_greedy=True, ignore_eos=True))
    if tp.rank == 0:
        q.put((tp.replica, out))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_dp2_tp2_world_split(tmp_path):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    d = str(tmp_path / "gptj")
    save_hf_model("gptj", d, vocab=101)
    ref = LLMEngine(build_model(d, None, "fp32", "cpu"), max_num_seqs=8, block_size=4, num_blocks=128)
    want = ref.generate(_prompts(6), SamplingParams(max_new_tokens=6, is_greedy=True, ignore_eos=True))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, port, d, q)) for r in range(4)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=300) for _ in range(2))
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    assert [p.exitcode for p in procs] == [0] * 4
    assert res[0] == want[0::2] and res[1] == want[1::2]
