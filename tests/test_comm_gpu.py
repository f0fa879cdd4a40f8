"""Native RCCL communicator (csrc/comm.cpp) on the one-GPU box.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so these tests run a ONE-rank
communicator: they check the binding (dtype codes, pointers, streams), that the calls are captured into
HIP graphs and replay, and the TP engine end to end with the native data plane in its graphs. They are
capture smoke tests - a one-rank all-reduce moves no data. The multi-rank behaviour (sums over xGMI,
per-collective latency) is measured by bench.py's comm probe in the driver's multi-GPU run
(``comm_probe`` in the bench JSON) and rehearsed on CPU by tests/test_bench_dist.py.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from llmss_amd import _native

    C = _native()
    c = C.RcclComm(C.rccl_unique_id(), 1, 0, torch.cuda.current_device())
    yield c
    c.destroy()


def _code(t):
    from llmss_amd import _native

    return _native().rccl_dtypes[str(t.dtype).replace("torch.", "")]


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.int64])
def test_single_rank_collectives(comm, dtype):
    x = (torch.arange(1000, device="cuda") % 97).to(dtype)
    ref = x.clone()
    comm.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), _code(x), _st())
    out = torch.empty_like(x)
    comm.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), _code(x), _st())
    comm.broadcast(x.data_ptr(), x.numel(), _code(x), 0, _st())
    torch.cuda.synchronize()
    assert torch.equal(x, ref) and torch.equal(out, ref)
    assert comm.async_error() == ""


def test_collective_inside_graph_replays(comm):
    """An out-of-place all-gather (one rank: a device copy) captured into a graph reads the CURRENT input on
    every replay - the captured node is live, not a recording of the capture-time values."""
    x = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), _code(x), _st())
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        comm.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), _code(x), _st())
        comm.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), _code(x), _st())
    for v in (1.0, 2.5, -3.0):
        x.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert bool((out == v).all())


def test_tp_engine_with_native_comm_in_graphs(comm):
    """TP=2 shard plan with the native communicator as its data plane: every row-parallel all-reduce and
    the candidate gather go through RcclComm, inside the captured decode graphs; graphs == eager."""
    from llmss_amd.engine import LLMEngine, SamplingParams
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights
    from llmss_amd.parallel.dist import TPGroup

    class OneRankNative(TPGroup):  # the comm has one rank; the shard plan claims 2 (gather = 2 copies)
        def all_gather_last_dim(self, t):
            t = t.contiguous()
            out = torch.empty_like(t)
            self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), self._code(t), _st())
            return torch.cat([out, out], -1)

        def all_reduce_int(self, v, op="min"):
            return int(v)

        def check_consistent(self, what, fp):
            pass

        def all_gather_object(self, obj):
            return [obj, obj]

    tp = OneRankNative(0, 2, comm=comm)
    assert tp.backend == "rccl-native" and not tp.host_staged
    cfg = get_preset("tiny-llama", hidden_size=256, num_heads=4, num_kv_heads=2, head_dim=64, rotary_dim=64,
                     intermediate_size=512, max_position_embeddings=256)
    m = DecoderLM(cfg, random_weights(cfg, 2, 0, device="cuda", dtype=torch.bfloat16, seed=3, std=0.05), tp)
    prompts = [[int(x) for x in torch.randint(0, cfg.vocab_size, (n,))] for n in (5, 17, 33)]
    sp = SamplingParams(max_new_tokens=12, is_greedy=True, ignore_eos=True)
    e_graph = LLMEngine(m, max_num_seqs=4, block_size=16, use_graphs=True, autotune=False)
    assert e_graph.use_graphs and len(e_graph.graphs) > 0
    out_g = e_graph.generate(prompts, sp)
    del e_graph
    e_eager = LLMEngine(m, max_num_seqs=4, block_size=16, use_graphs=False, autotune=False)
    assert e_eager.generate(prompts, sp) == out_g


def test_decode_overlap_ab_at_capture(comm, monkeypatch):
    """The capture-time A/B of the two-micro-batch decode schedule runs on a native-comm TP group, records
    both timings, keeps one graph per bucket, and whatever it keeps decodes exactly like eager."""
    from llmss_amd.engine import LLMEngine, SamplingParams
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights
    from llmss_amd.parallel.dist import TPGroup

    class OneRankNative(TPGroup):
        def all_gather_last_dim(self, t):
            t = t.contiguous()
            out = torch.empty_like(t)
            self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), self._code(t), _st())
            return torch.cat([out, out], -1)

        def all_reduce_int(self, v, op="min"):
            return int(v)

        def check_consistent(self, what, fp):
            pass

        def all_gather_object(self, obj):
            return [obj, obj]

    monkeypatch.setenv("LLMSS_TBO_AUTO_MIN", "16")
    monkeypatch.setenv("LLMSS_TP_RSAG", "0")  # the one-rank stand-in's reduce-scatter is no TP=2 reduce-scatter
    monkeypatch.setenv("LLMSS_TP_COL", "0")  # A/B of the micro-batch schedule alone (col: its own test below)
    tp = OneRankNative(0, 2, comm=comm)
    cfg = get_preset("tiny-llama", hidden_size=256, num_heads=4, num_kv_heads=2, head_dim=64, rotary_dim=64,
                     intermediate_size=512, max_position_embeddings=256)
    m = DecoderLM(cfg, random_weights(cfg, 2, 0, device="cuda", dtype=torch.bfloat16, seed=5, std=0.05), tp)
    prompts = [[int(x) for x in torch.randint(0, cfg.vocab_size, (n,))] for n in range(3, 23)]
    sp = SamplingParams(max_new_tokens=10, is_greedy=True, ignore_eos=True)
    e = LLMEngine(m, max_num_seqs=24, block_size=16, use_graphs=True, autotune=False, graph_buckets=[1, 8, 16, 24])
    assert e._tbo_cands == [16, 24] and set(e.stats["schedule_ab_ms"]) >= {"16c", "24c"}
    assert all(set(v) == {"one", "tbo"} for v in e.stats["schedule_ab_ms"].values())
    out_g = e.generate(prompts, sp)
    del e
    e2 = LLMEngine(m, max_num_seqs=24, block_size=16, use_graphs=False, autotune=False)
    assert e2.generate(prompts, sp) == out_g


def _graph_node_types(g):
    """Types of the nodes of a captured torch CUDAGraph (keep_graph=True), read with hipGraphGetNodes."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    graph = ctypes.c_void_p(g.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * max(1, n.value))()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
    types = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        assert hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) == 0
        types.append(t.value)
    return types


def test_captured_collectives_are_graph_nodes(comm):
    """'capture succeeded' is not the check. Out-of-place all-gather / all-reduce /
    reduce-scatter on the native communicator captured into one graph leave one node each (a one-rank
    collective is a device copy: memcpy or kernel nodes, never an empty graph), and the replay moves the
    CURRENT inputs."""
    xs = [torch.zeros(4096, dtype=dt, device="cuda") for dt in (torch.bfloat16, torch.float32, torch.bfloat16)]
    outs = [torch.empty_like(x) for x in xs]
    ops = [lambda: comm.all_gather(xs[0].data_ptr(), outs[0].data_ptr(), xs[0].numel(), _code(xs[0]), _st()),
           lambda: comm.all_reduce(xs[1].data_ptr(), outs[1].data_ptr(), xs[1].numel(), _code(xs[1]), _st()),
           lambda: comm.reduce_scatter(xs[2].data_ptr(), outs[2].data_ptr(), xs[2].numel(), _code(xs[2]), _st())]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for op in ops:
            op()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for op in ops:
            op()
    types = _graph_node_types(g)
    # hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset, 5 empty; one-rank collectives copy
    assert len([t for t in types if t in (0, 1)]) >= len(ops), types
    g.instantiate()
    for v in (3.0, 7.0):
        for x in xs:
            x.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert all(bool((o == v).all()) for o in outs)


def test_rccl_setting_probe_one_rank(monkeypatch):
    """The start-up probe of RCCL protocol / algorithm settings (parallel/dist.py _tune_native_comm) builds a
    communicator per candidate environment, times the graph-replayed all-reduce on each, keeps one communicator
    that still works and restores the environment (one rank: the mechanism; the multi-rank timing runs in the
    driver's multi-GPU bench and lands in its runtime record)."""
    import os
    import socket

    import torch.distributed as dist

    from llmss_amd import _native
    from llmss_amd.parallel import dist as D

    C = _native()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    monkeypatch.delenv("NCCL_PROTO", raising=False)
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        c0 = C.RcclComm(C.rccl_unique_id(), 1, 0, torch.cuda.current_device())
        kept = D._tune_native_comm(c0, 0, 1, 1 << 20)
        info = D.RCCL_TUNE_INFO
        assert info["bytes"] == 1 << 20 and set(info["us"]) == {n for n, _ in D.RCCL_CANDIDATES}
        assert info["kept"] in info["us"] and info["us"]["default"] > 0
        assert os.environ.get("NCCL_PROTO") == info["env"].get("NCCL_PROTO")
        x = torch.arange(64, dtype=torch.float32, device="cuda")
        out = torch.empty_like(x)
        kept.all_gather(x.data_ptr(), out.data_ptr(), x.numel(), C.rccl_dtypes["float32"], _st())
        torch.cuda.synchronize()
        assert torch.equal(out, x)
        kept.destroy()
    finally:
        dist.destroy_process_group()
        os.environ.pop("NCCL_PROTO", None)
        os.environ.pop("NCCL_ALGO", None)


def test_rccl_init_deadline_without_peer():
    """Bounded communicator init (csrc/comm.cpp): a 2-rank communicator whose second rank
    never arrives raises at the deadline (non-blocking ncclCommInitRankConfig polled, then ncclCommAbort) instead
    of blocking forever; a 1-rank communicator still initialises and reports its set-up time."""
    import time

    from llmss_amd import _native

    C = _native()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="timed out"):
        C.RcclComm(C.rccl_unique_id(), 2, 0, torch.cuda.current_device(), 3.0)
    assert time.monotonic() - t0 < 60
    c = C.RcclComm(C.rccl_unique_id(), 1, 0, torch.cuda.current_device(), 30.0)
    assert 0 <= c.init_seconds < 30
    x = torch.ones(16, device="cuda")
    c.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), _code(x), _st())
    torch.cuda.synchronize()
    assert bool((x == 1).all())
    c.destroy()


def test_col_schedule_ab_at_capture(comm, monkeypatch):
    """the column-chunked decode schedule (DecoderLM._reduce_cols: each row-parallel output
    as weight-row slices whose all-reduces run on the comm stream beside the next slice's GEMM) is a fourth
    capture-time A/B candidate on a native-comm TP group: both timings recorded, one graph kept per bucket, and
    what it keeps decodes exactly like eager (one-rank stand-in for TP=2, as the micro-batch A/B test)."""
    from llmss_amd.engine import LLMEngine, SamplingParams
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights
    from llmss_amd.parallel.dist import TPGroup

    class OneRankNative(TPGroup):
        def all_gather_last_dim(self, t):
            t = t.contiguous()
            out = torch.empty_like(t)
            self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), self._code(t), _st())
            return torch.cat([out, out], -1)

        def all_reduce_int(self, v, op="min"):
            return int(v)

        def check_consistent(self, what, fp):
            pass

        def all_gather_object(self, obj):
            return [obj, obj]

    monkeypatch.setenv("LLMSS_TBO_AUTO_MIN", "0")
    monkeypatch.setenv("LLMSS_TP_RSAG", "0")
    monkeypatch.setenv("LLMSS_TP_COL", "auto")
    tp = OneRankNative(0, 2, comm=comm)
    cfg = get_preset("tiny-llama", hidden_size=256, num_heads=4, num_kv_heads=2, head_dim=64, rotary_dim=64,
                     intermediate_size=512, max_position_embeddings=256)
    m = DecoderLM(cfg, random_weights(cfg, 2, 0, device="cuda", dtype=torch.bfloat16, seed=5, std=0.05), tp)
    prompts = [[int(x) for x in torch.randint(0, cfg.vocab_size, (n,))] for n in range(3, 23)]
    sp = SamplingParams(max_new_tokens=10, is_greedy=True, ignore_eos=True)
    m.col_min = 8
    e = LLMEngine(m, max_num_seqs=24, block_size=16, use_graphs=True, autotune=False, graph_buckets=[1, 8, 16, 24])
    # timed buckets 8 and 24 (LLMEngine._ab_buckets); 16 adopts the winner of its nearest timed bucket
    assert e._col_cands == [8, 16, 24] and set(e.stats["schedule_ab_ms"]) >= {"8c", "24c"}
    assert "16c" not in e.stats["schedule_ab_ms"]
    assert all(set(v) == {"one", "col"} for v in e.stats["schedule_ab_ms"].values())
    out_g = e.generate(prompts, sp)
    del e
    e2 = LLMEngine(m, max_num_seqs=24, block_size=16, use_graphs=False, autotune=False)
    assert e2.generate(prompts, sp) == out_g
