"""Failure detection in the serving driver: server-side deadlines, a follower that
dies mid-generation (every in-flight request must fail, not hang), a leader that disappears
(followers must notice through the heartbeat timeout), and the fault-injection hook."""
import os
import queue
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from helpers import save_hf_model


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("fail_llama"))
    save_hf_model("llama", d, vocab=101)
    return d


def test_deadline_aborts_request(ckpt):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.serving.driver import EngineDriver

    m = build_model(ckpt, None, "fp32", "cpu")
    drv = EngineDriver(LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=128, eos_token_id=None)).start()
    try:
        h = drv.submit([1, 2, 3], SamplingParams(max_new_tokens=10_000, is_greedy=True, ignore_eos=True),
                       deadline_s=0.0)
        assert h.wait(30)
        assert h.finish_reason == "deadline" and len(h.output_ids) < 10_000
        ok = drv.submit([4, 5], SamplingParams(max_new_tokens=3, is_greedy=True, ignore_eos=True))
        assert ok.wait(30) and ok.finish_reason == "length" and len(ok.output_ids) == 3
    finally:
        drv.stop()


def _worker(rank, world, port, ckpt, role, q, ctrl="shm"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LLMSS_CTRL=ctrl)
    torch.set_num_threads(1)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed
    from llmss_amd.serving.driver import EngineDriver, FaultSpec

    tp, r, w = initialize_distributed(backend="gloo", timeout_s=20)
    m = build_model(ckpt, tp, "fp32", "cpu")
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64, eos_token_id=None)
    fault = FaultSpec(1, 3, "exit") if role == "follower_crash" else None
    drv = EngineDriver(eng, heartbeat_s=0.2, leader_timeout_s=5.0, fault=fault).start()
    if role == "follower_crash":
        if r == 0:
            h = drv.submit([1, 2, 3, 4], SamplingParams(max_new_tokens=50, is_greedy=True, ignore_eos=True))
            done = h.wait(90)
            q.put(("leader", done, h.finish_reason, len(h.output_ids), h.error))
            later = drv.submit([5, 6], SamplingParams(max_new_tokens=2, is_greedy=True))
            q.put(("later", later.wait(5), later.finish_reason))
            q.close()
            q.join_thread()  # flush the queue's feeder thread before the hard exit
            os._exit(0)
        drv._thread.join(120)  # rank 1 exits inside the driver (os._exit(17)) at step 3
        os._exit(0)
    else:  # leader_loss
        if r == 0:
            time.sleep(1.5)  # a few idle heartbeats
            os._exit(0)  # leader vanishes without a word
        t0 = time.time()
        drv._thread.join(60)
        q.put(("follower", drv.error is not None, time.time() - t0, str(drv.error)[:200], drv.ctrl))
        q.close()
        q.join_thread()
        os._exit(0)


def _spawn(world, ckpt, role, ctrl="shm"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ckpt, role, q, ctrl)) for r in range(world)]
    for p in procs:
        p.start()
    return procs, q


def _drain(q, n, timeout):
    out, t0 = [], time.time()
    while len(out) < n and time.time() - t0 < timeout:
        try:
            out.append(q.get(timeout=1))
        except queue.Empty:
            pass
    return out


@pytest.mark.parametrize("ctrl", ["shm", "gloo"])
def test_follower_crash_fails_inflight_requests(ckpt, ctrl):
    procs, q = _spawn(2, ckpt, "follower_crash", ctrl)
    try:
        res = {r[0]: r for r in _drain(q, 2, 150)}
        assert "leader" in res, res
        _, done, reason, ntok, err = res["leader"]
        assert done and reason == "error" and ntok < 50 and err
        assert res["later"][1] and res["later"][2] == "error"  # a failed driver refuses new work
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert procs[1].exitcode == 17  # the injected exit


@pytest.mark.parametrize("ctrl", ["shm", "gloo"])
def test_leader_loss_detected_by_follower(ckpt, ctrl):
    """gloo: the heartbeat timeout (leader_timeout_s = 5 s) ends the follower. shm ring: the follower sees
    the leader's process gone while it waits for the next record (no timeout needed)."""
    procs, q = _spawn(2, ckpt, "leader_loss", ctrl)
    try:
        res = _drain(q, 1, 120)
        assert res and res[0][0] == "follower", res
        _, errored, waited, msg, mode = res[0]
        assert errored and waited < 60, res
        assert mode == ("shm-ring" if ctrl == "shm" else "gloo"), res
        if ctrl == "shm":
            assert "producer process died" in msg, res
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()


class _RendezvousComm:
    """Stand-in for the native RcclComm's bounded init (csrc/comm.cpp): every rank announces itself in a shared
    directory and waits for all ``nranks`` peers until ``timeout_s``, then raises like the native deadline."""

    def __init__(self, root, timeout_s):
        self.root, self.timeout_s = root, timeout_s

    def __call__(self, uid, nranks, rank, device):
        d = os.path.join(self.root, uid.hex()[:16])
        os.makedirs(d, exist_ok=True)
        open(os.path.join(d, str(rank)), "w").close()
        t0 = time.monotonic()
        while len(os.listdir(d)) < nranks:
            if time.monotonic() - t0 > self.timeout_s:
                raise RuntimeError(f"RCCL ncclCommInitRankConfig: timed out after {self.timeout_s} s waiting for "
                                   "the peer ranks (communicator aborted)")
            time.sleep(0.01)
        return object()


def _init_worker(rank, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LLMSS_FAULT_INJECT="1:rccl_init:skip")
    import torch.distributed as dist

    from llmss_amd.parallel.dist import _native_comm

    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device = lambda *a: None  # no GPU here: the device step is stubbed (tests/test_capture_agreement.py)
    torch.cuda.synchronize = lambda *a: None
    torch.cuda.current_device = lambda: 0
    t0 = time.monotonic()
    err = ""
    try:
        _native_comm(rank, 1, 2, make_comm=_RendezvousComm(root, 3.0), unique_id=lambda: os.urandom(128))
    except RuntimeError as e:
        err = str(e)
    el = time.monotonic() - t0
    ok = torch.tensor([0 if err else 1], dtype=torch.int32)  # the caller's agreement (initialize_distributed)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    q.put((rank, el, err, int(ok[0])))
    dist.destroy_process_group()


def test_rccl_init_bounded_when_a_peer_never_joins(tmp_path):
    """rank 1 passes the pre-init agreement and then never joins the communicator init
    (fault-injected, as a peer that died). Rank 0's bounded init raises at its deadline instead of blocking, and
    both ranks then agree on the failure over gloo (the native deadline itself: tests/test_comm_gpu.py)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_init_worker, args=(r, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = {r: (el, err, ok) for r, el, err, ok in (q.get(timeout=120) for _ in range(2))}
        for p in procs:
            p.join(30)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    el0, err0, ok0 = res[0]
    assert "timed out" in err0 and 2.5 < el0 < 30, res[0]
    assert "injected" in res[1][1]
    assert ok0 == 0 and res[1][2] == 0
