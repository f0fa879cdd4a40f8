"""Serving path on CPU: broker semantics (in-memory and RESP over TCP), the HTTP producer, the
TP driver + consumer, gRPC (direct and via the broker), request/response correlation under
concurrent clients (reference quirk Q11), and reference-format interoperability."""
import concurrent.futures as cf
import json
import os
import threading
import time

import grpc
import pytest
import torch

from helpers import save_hf_model
from llmss_amd.engine import LLMEngine, build_model
from llmss_amd.engine.sampling import SamplingParams
from llmss_amd.serving.broker import PQUEUE, SQUEUE, MemoryBroker, MiniRedisServer, RedisBroker, reply_key
from llmss_amd.serving.consumer import Consumer
from llmss_amd.serving.driver import EngineDriver
from llmss_amd.serving.grpc_api import BrokerServicer, EngineServicer, GenerateRequest, Stub, serve
from llmss_amd.utils.tokenizer import encode, load_tokenizer


@pytest.mark.parametrize("kind", ["memory", "resp"])
def test_broker_list_semantics(kind):
    srv = None
    if kind == "memory":
        b = MemoryBroker()
    else:
        srv = MiniRedisServer().start()
        b = RedisBroker(srv.host, srv.port)
        assert b.ping() == "PONG"
    assert b.llen("q") == 0 and b.rpop("q") is None
    b.lpush("q", "a")
    b.lpush("q", "b")
    b.lpush("q", "ü-unicode")
    assert b.llen("q") == 3
    assert b.rpop("q") == "a"  # LPUSH + RPOP = FIFO like the reference queues
    assert b.brpop("q", 1) == "b"
    assert b.rpop("q") == "ü-unicode"
    t0 = time.time()
    assert b.brpop("q", 0.3) is None and time.time() - t0 >= 0.25
    threading.Timer(0.2, lambda: b.lpush("q", "late")).start()
    assert b.brpop("q", 5) == "late"
    if srv:
        b.close()
        srv.stop()


def test_memory_broker_wakes_each_key_and_leaves_no_empty_keys():
    """64 blocked pops on 64 reply keys: each push wakes its own key's waiter (per-key conditions, not one shared
    condition that every push broadcast to all waiters), every waiter gets its own value, several values on one key
    go to several waiters, and emptied lists / waiter records are deleted (one-shot reply keys leave nothing)."""
    b = MemoryBroker()
    got = {}

    def wait(i):
        got[i] = b.brpop(f"squeue:{i}", 10)

    ths = [threading.Thread(target=wait, args=(i,)) for i in range(64)]
    for t in ths:
        t.start()
    deadline = time.time() + 10
    while sum(w[1] for w in list(b._waiters.values())) < 64 and time.time() < deadline:
        time.sleep(0.01)
    assert len(b._waiters) == 64
    b.pipeline([("LPUSH", f"squeue:{i}", f"v{i}") for i in range(64)])
    for t in ths:
        t.join(10)
    assert got == {i: f"v{i}" for i in range(64)}
    assert not b._lists and not b._waiters
    # three waiters, one key, three values; brpoplpush moves and wakes the destination's waiter
    out = []
    ths = [threading.Thread(target=lambda: out.append(b.brpop("k", 10))) for _ in range(3)]
    for t in ths:
        t.start()
    for v in ("a", "b", "c"):
        b.lpush("k", v)
    for t in ths:
        t.join(10)
    assert sorted(out) == ["a", "b", "c"] and not b._lists
    b.lpush("src", "x")
    assert b.brpoplpush("src", "proc", 1) == "x" and b.lrange("proc", 0, -1) == ["x"]
    assert b.lrem("proc", 0, "x") == 1 and not b._lists and b.llen("proc") == 0
    t0 = time.time()
    assert b.brpop("none", 0.2) is None and 0.15 < time.time() - t0 < 5 and not b._waiters


@pytest.fixture(scope="module")
def model_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("gpt2tok"))
    save_hf_model("gpt2", d, vocab=101, with_tokenizer=True)
    return d


@pytest.fixture(scope="module")
def driver(model_dir):
    m = build_model(model_dir, None, "fp32", "cpu")
    tok = load_tokenizer(model_dir, m.cfg.vocab_size)
    eng = LLMEngine(m, max_num_seqs=8, block_size=4, num_blocks=256, eos_token_id=None)
    drv = EngineDriver(eng).start()
    yield drv, tok, m
    drv.stop()


def _offline(m, tok, prompt, n):
    from llmss_amd.utils.tokenizer import encode

    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=128, eos_token_id=None)
    return tok.decode(eng.generate([encode(tok, prompt)], SamplingParams(max_new_tokens=n, is_greedy=True))[0])


def test_driver_concurrent_requests(driver):
    drv, tok, m = driver
    from llmss_amd.utils.tokenizer import encode

    prompts = ["hello world", "this is", "tiny corpus for", "an offline tokenizer", "hello"]
    hs = [drv.submit(encode(tok, p), SamplingParams(max_new_tokens=6 + i, is_greedy=True)) for i, p in enumerate(prompts)]
    for i, (h, p) in enumerate(zip(hs, prompts)):
        assert h.wait(60)
        assert len(h.output_ids) == 6 + i
        assert tok.decode(h.output_ids) == _offline(m, tok, p, 6 + i)


def test_producer_consumer_http(driver):
    from fastapi.testclient import TestClient

    from llmss_amd.serving.producer import create_app

    drv, tok, m = driver
    srv = MiniRedisServer().start()
    consumer = Consumer(drv, tok, RedisBroker(srv.host, srv.port), poll_timeout=0.2).start()
    client = TestClient(create_app(RedisBroker(srv.host, srv.port), timeout_s=60))
    prompts = [f"hello world {i}" for i in range(6)]

    def call(p):
        r = client.post("/generate", json={"prompt": p, "max_new_tokens": 5, "is_greedy": True, "temperature": 1.0,
                                            "top_p": 0.95, "top_k": 50})
        assert r.status_code == 200
        return p, r.json()

    with cf.ThreadPoolExecutor(6) as ex:
        results = list(ex.map(call, prompts))
    for p, body in results:
        assert body["prompt"] == p  # correlation: every client gets its own reply
        assert body["continuation"] == _offline(m, tok, p, 5)
    assert client.get("/health").json() == {"status": "ok"}
    assert "llmss_producer_completed 6" in client.get("/metrics").text
    consumer.stop()
    srv.stop()


def test_consumer_survives_a_broker_restart(driver):
    """The consumer's intake reconnects when the broker goes away and comes back on the same port (a Redis
    restart): the request pushed after the restart is served, and the intake thread never dies."""
    drv, tok, m = driver
    srv = MiniRedisServer().start()
    port = srv.port
    consumer = Consumer(drv, tok, RedisBroker("127.0.0.1", port), poll_timeout=0.05, durable=False).start()
    try:
        time.sleep(0.2)
        srv.stop()
        time.sleep(0.3)  # the intake sees the connection drop and backs off
        assert consumer._intake.is_alive()
        srv = MiniRedisServer("127.0.0.1", port).start()
        b = RedisBroker("127.0.0.1", port)
        b.lpush(PQUEUE, json.dumps({"prompt": "hello", "max_new_tokens": 3, "is_greedy": True, "temperature": 1.0,
                                    "top_p": 0.95, "top_k": 50, "request_id": "after"}))
        d = json.loads(b.brpop(reply_key("after"), 30))
        assert d["continuation"] == _offline(m, tok, "hello", 3)
    finally:
        consumer.stop()
        srv.stop()


def test_reference_format_interop(driver):
    """A reference producer pushes a request without request_id and pops plain 'squeue'."""
    drv, tok, m = driver
    b = MemoryBroker()
    consumer = Consumer(drv, tok, b, poll_timeout=0.2).start()
    b.lpush(PQUEUE, json.dumps({"prompt": "hello", "max_new_tokens": 4, "is_greedy": True, "temperature": 1.0,
                                "top_p": 0.95, "top_k": 50}))
    msg = b.brpop(SQUEUE, 30)
    assert msg is not None
    d = json.loads(msg)
    assert set(d) == {"prompt", "continuation"} and d["prompt"] == "hello"
    # invalid request -> error reply, consumer keeps serving
    b.lpush(PQUEUE, json.dumps({"prompt": "x", "max_new_tokens": 0, "is_greedy": True, "temperature": 1.0,
                                "top_p": 0.95, "top_k": 50, "request_id": "bad"}))
    assert "error" in json.loads(b.brpop(reply_key("bad"), 30))
    consumer.stop()


def test_grpc_direct_and_broker(driver):
    drv, tok, m = driver
    server = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
    ch = grpc.insecure_channel(f"127.0.0.1:{server.bound_port}")
    stub = Stub(ch)
    r = stub.Generate(GenerateRequest(prompt="hello world", max_new_tokens=5, is_greedy=True), timeout=60)
    assert r.continuation == _offline(m, tok, "hello world", 5) and len(r.token_ids) == 5
    toks = list(stub.GenerateStream(GenerateRequest(prompt="hello world", max_new_tokens=5, is_greedy=True),
                                    timeout=60))
    assert toks[-1].finished and "".join(t.text for t in toks[:-1]) == r.continuation
    with pytest.raises(grpc.RpcError) as e:
        stub.Generate(GenerateRequest(prompt="x", max_new_tokens=5, temperature=1.5), timeout=10)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    assert json.loads(stub.Stats(__import__("llmss_amd.serving.grpc_api", fromlist=["StatsRequest"]).StatsRequest(),
                                 timeout=10).json)["tokens"] > 0

    # gRPC front-end on the pub/sub broker, concurrent clients
    b = MemoryBroker()
    consumer = Consumer(drv, tok, b, poll_timeout=0.2).start()
    fe = serve(BrokerServicer(b), port=0, host="127.0.0.1")
    stub2 = Stub(grpc.insecure_channel(f"127.0.0.1:{fe.bound_port}"))
    prompts = [f"tiny {i}" for i in range(8)]
    with cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda p: stub2.Generate(GenerateRequest(prompt=p, max_new_tokens=4, is_greedy=True),
                                                    timeout=60), prompts))
    for p, o in zip(prompts, outs):
        assert o.prompt == p and o.continuation == _offline(m, tok, p, 4)
    consumer.stop()
    fe.stop(0)
    server.stop(0)


def test_broker_grpc_stream_streams_tokens(driver):
    """VERDICT r2 missing 5: GenerateStream on the pub/sub path yields the tokens as the engine samples them
    (one broker message per engine step), not one message after the whole reply."""
    drv, tok, m = driver
    b = MemoryBroker()
    consumer = Consumer(drv, tok, b, poll_timeout=0.2).start()
    fe = serve(BrokerServicer(b), port=0, host="127.0.0.1")
    stub = Stub(grpc.insecure_channel(f"127.0.0.1:{fe.bound_port}"))
    req = GenerateRequest(prompt="hello world", max_new_tokens=6, is_greedy=True, request_id="s1")
    toks = list(stub.GenerateStream(req, timeout=60))
    assert toks[-1].finished and toks[-1].finish_reason == "length"
    ids = [t.token_id for t in toks[:-1]]
    assert len(ids) == 6
    assert tok.decode(ids) == _offline(m, tok, "hello world", 6)
    assert "".join(t.text for t in toks[:-1]) == _offline(m, tok, "hello world", 6)
    consumer.stop()
    fe.stop(0)


def test_durable_queue_requeues_after_consumer_crash(driver):
    """VERDICT r2 missing 7: a request popped by a consumer that then died stays in its processing list; a
    consumer restarted with the same id re-queues and serves it, and acknowledges every reply."""
    from llmss_amd.serving.consumer import processing_key

    drv, tok, m = driver
    b = MemoryBroker()
    body = json.dumps({"prompt": "hello", "max_new_tokens": 4, "is_greedy": True, "temperature": 1.0,
                       "top_p": 0.95, "top_k": 50, "request_id": "lost"})
    b.lpush(PQUEUE, body)
    assert b.brpoplpush(PQUEUE, processing_key("c7"), 1) == body  # the dead consumer's pop
    assert b.llen(PQUEUE) == 0 and b.llen(processing_key("c7")) == 1
    consumer = Consumer(drv, tok, b, poll_timeout=0.2, consumer_id="c7").start()
    msg = b.brpop(reply_key("lost"), 60)
    assert msg is not None and json.loads(msg)["continuation"] == _offline(m, tok, "hello", 4)
    assert consumer.requeued == 1
    for _ in range(100):
        if b.llen(processing_key("c7")) == 0:
            break
        time.sleep(0.05)
    assert b.llen(processing_key("c7")) == 0  # acknowledged
    consumer.stop()


def test_durable_intake_recovers_requests_of_a_failed_batch_pop(driver):
    """the connection drops after the server ran part of the intake's batch pop. The requests those pops
    moved into the processing list are resubmitted at once (no restart needed), none is served twice, every one is
    answered and acknowledged."""
    from llmss_amd.serving.consumer import processing_key

    drv, tok, m = driver

    class DropAfter2(MemoryBroker):
        fail = True

        def pipeline(self, cmds):
            if self.fail and cmds and cmds[0][0] == "RPOPLPUSH":
                self.fail = False
                super().pipeline(cmds[:2])  # ran on the server, replies lost
                raise ConnectionError("connection reset mid-pipeline")
            return super().pipeline(cmds)

    b = DropAfter2()
    n = 5
    for i in range(n):
        b.lpush(PQUEUE, json.dumps({"prompt": f"drop {i}", "max_new_tokens": 3, "is_greedy": True, "temperature": 1.0,
                                    "top_p": 0.95, "top_k": 50, "request_id": f"d{i}"}))
    consumer = Consumer(drv, tok, b, poll_timeout=0.2, consumer_id="cd").start()
    try:
        for i in range(n):
            msg = b.brpop(reply_key(f"d{i}"), 60)
            assert msg is not None and json.loads(msg)["continuation"] == _offline(m, tok, f"drop {i}", 3)
        assert not b.fail  # the failure really happened
        for _ in range(100):
            if b.llen(processing_key("cd")) == 0:
                break
            time.sleep(0.05)
        assert b.llen(processing_key("cd")) == 0
        time.sleep(0.3)
        assert consumer.served == n and all(b.llen(reply_key(f"d{i}")) == 0 for i in range(n))  # nothing twice
    finally:
        consumer.stop()


def test_redis_broker_list_commands():
    """BRPOPLPUSH / LREM / LRANGE over RESP against the embedded server (Redis semantics)."""
    srv = MiniRedisServer().start()
    b = RedisBroker(srv.host, srv.port)
    for v in ("a", "b", "a", "c"):
        b.lpush("k", v)  # k = [c, a, b, a]
    assert b.lrange("k", 0, -1) == ["c", "a", "b", "a"]
    assert b.brpoplpush("k", "p", 1) == "a" and b.lrange("p", 0, -1) == ["a"]
    assert b.lrem("k", 0, "a") == 1 and b.lrange("k", 0, -1) == ["c", "b"]
    assert b.brpoplpush("empty", "p", 0.1) is None
    srv.stop()


def test_redis_rotation_onto_the_same_key_with_parked_pops():
    """Two BRPOPLPUSH q -> q pops park on an empty list; one push serves both (the first pop's move onto q serves
    the second from inside the first's wake-up), as Redis rotates a list onto itself. The server stays up."""
    srv = MiniRedisServer().start()
    try:
        got = []
        ts = [threading.Thread(target=lambda: got.append(RedisBroker(srv.host, srv.port).brpoplpush("q", "q", 5)))
              for _ in range(2)]
        for t in ts:
            t.start()
        time.sleep(0.3)
        b = RedisBroker(srv.host, srv.port)
        b.lpush("q", "x")
        for t in ts:
            t.join(10)
        assert got == ["x", "x"] and b.lrange("q", 0, -1) == ["x"]
        assert b.pipeline([("PING",)]) == ["PONG"]
    finally:
        srv.stop()


@pytest.mark.parametrize("kind", ["memory", "resp"])
def test_broker_pipeline(kind):
    """Pipelined commands run in order with one reply each; an error reply sits in its slot and the commands after
    it still run; RPOPLPUSH on an empty list is None (the consumer's batched intake)."""
    srv = MiniRedisServer().start() if kind == "resp" else None
    b = RedisBroker(srv.host, srv.port) if srv else MemoryBroker()
    try:
        r = b.pipeline([("LPUSH", "q", "a"), ("LPUSH", "q", "b"), ("RPOPLPUSH", "q", "p"), ("NOPE", "x"),
                        ("RPOPLPUSH", "q", "p"), ("RPOPLPUSH", "q", "p"), ("LREM", "p", 1, "a"), ("LLEN", "p")])
        assert r[:3] == [1, 2, "a"] and isinstance(r[3], Exception)
        assert r[4:] == ["b", None, 1, 1]
        assert b.lrange("p", 0, -1) == ["b"] and b.pipeline([]) == []
    finally:
        if srv:
            srv.stop()


def test_consumer_takes_a_queued_burst_in_one_step(driver):
    """Requests already queued when the consumer wakes are popped together (one blocking pop plus one pipeline of
    non-blocking pops) and admitted together (one prefill step; two if the engine loop wakes between the submits);
    every one is answered and acknowledged."""
    from llmss_amd.serving.consumer import processing_key

    drv, tok, m = driver
    srv = MiniRedisServer().start()
    b = RedisBroker(srv.host, srv.port)
    n = 6
    for i in range(n):
        b.lpush(PQUEUE, json.dumps({"prompt": f"burst {i}", "max_new_tokens": 3, "is_greedy": True,
                                    "temperature": 1.0, "top_p": 0.95, "top_k": 50, "request_id": f"b{i}"}))
    before = drv.engine.stats["prefill_steps"]
    consumer = Consumer(drv, tok, RedisBroker(srv.host, srv.port), poll_timeout=0.2, consumer_id="cb").start()
    try:
        for i in range(n):
            msg = b.brpop(reply_key(f"b{i}"), 60)
            assert msg is not None and json.loads(msg)["continuation"] == _offline(m, tok, f"burst {i}", 3)
        assert drv.engine.stats["prefill_steps"] - before <= 2  # one, or two if the engine woke between submits
        for _ in range(100):
            if b.llen(processing_key("cb")) == 0:
                break
            time.sleep(0.05)
        assert b.llen(processing_key("cb")) == 0 and consumer.served == n
    finally:
        consumer.stop()
        srv.stop()


def test_admission_window_batches_a_burst(driver):
    """A burst of concurrent submissions to an idle driver is admitted in one prefill step."""
    drv, tok, m = driver
    eng = drv.engine
    before = eng.stats["prefill_steps"]
    hs = []

    def sub(i):
        time.sleep(0.0005 * i)
        hs.append(drv.submit(encode(tok, f"burst {i}"), SamplingParams(max_new_tokens=3, is_greedy=True)))

    old = drv.batch_window_s
    drv.batch_window_s = 0.1  # generous: the suite runs under parallel load (pytest -n)
    try:
        with cf.ThreadPoolExecutor(6) as ex:
            list(ex.map(sub, range(6)))
        assert all(h.wait(60) for h in hs)
    finally:
        drv.batch_window_s = old
    assert eng.stats["prefill_steps"] - before == 1


def test_grpc_burst_lands_in_one_admission_step(model_dir):
    """The engine servicer runs on a grpc.aio server (coroutine handlers, no thread per in-flight request), and a
    burst of concurrent requests arriving while the engine is idle is admitted in ONE step (the driver's admission
    window), bursts after bursts included (the last step of a burst may leave a speculative decode step in flight)."""
    import concurrent.futures as cf

    from llmss_amd.serving.grpc_api import AioServer

    m = build_model(model_dir, None, "fp32", "cpu")
    tok = load_tokenizer(model_dir, m.cfg.vocab_size)
    eng = LLMEngine(m, max_num_seqs=8, block_size=4, num_blocks=256, eos_token_id=None)
    drv = EngineDriver(eng)
    drv.batch_window_s = 0.05  # CPU test box: generous gap between arrivals
    drv.start()
    server = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
    try:
        assert isinstance(server, AioServer)
        stub = Stub(grpc.insecure_channel(f"127.0.0.1:{server.bound_port}"))
        with cf.ThreadPoolExecutor(8) as ex:
            for burst in range(3):
                reqs = [GenerateRequest(prompt_token_ids=[1 + i, 2, 3, 4 + burst], max_new_tokens=6, is_greedy=True,
                                        ignore_eos=True) for i in range(8)]
                outs = list(ex.map(lambda r: stub.Generate(r, timeout=60), reqs))
                assert all(len(o.token_ids) == 6 for o in outs)
        assert drv.stats["admit_steps"] == 3, drv.stats
        assert drv.stats["admit_window_reqs"] == 24
    finally:
        server.stop(0).wait(10)
        drv.stop()


def test_stream_sink_batches_one_call_per_step(driver):
    """Handle.sink: the tokens of all streams sharing a sink arrive as ONE call per engine step, each stream's
    tokens in order and its end marker (None) after its last token (the gRPC stream servicer's hand-off)."""
    import threading

    from llmss_amd.utils.tokenizer import encode

    drv, tok, m = driver
    calls, lock = [], threading.Lock()

    def sink(items):
        with lock:
            calls.append(list(items))

    prompts = ["hello world", "this is", "tiny corpus for"]
    qs = [f"q{i}" for i in range(len(prompts))]
    hs = [drv.submit(encode(tok, p), SamplingParams(max_new_tokens=4 + i, is_greedy=True), sink=sink, sink_q=q)
          for i, (p, q) in enumerate(zip(prompts, qs))]
    for h in hs:
        assert h.wait(60)
    per_q = {q: [] for q in qs}
    for items in calls:
        for q, t in items:
            assert not per_q[q] or per_q[q][-1] is not None, "token after the end marker"
            per_q[q].append(t)
    for h, q, p, i in zip(hs, qs, prompts, range(len(prompts))):
        assert per_q[q][-1] is None and per_q[q][:-1] == h.output_ids
        assert tok.decode(h.output_ids) == _offline(m, tok, p, 4 + i)
    # fewer hand-offs than tokens: steps batch the streams together
    assert len(calls) < sum(len(v) for v in per_q.values())


def test_admission_window_closes_when_slots_are_full(model_dir):
    """A burst that fills every free sequence slot is admitted without waiting out the quiet period: nothing that
    arrives later could join that prefill step."""
    m = build_model(model_dir, None, "fp32", "cpu")
    tok = load_tokenizer(model_dir, m.cfg.vocab_size)
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=128, eos_token_id=None)
    drv = EngineDriver(eng)
    drv.batch_window_s = 0.5  # a full burst must not wait this long for more arrivals
    hs = [drv.submit(encode(tok, f"full {i}"), SamplingParams(max_new_tokens=3, is_greedy=True)) for i in range(4)]
    drv.start()
    try:
        assert all(h.wait(60) for h in hs)
        assert drv.stats["admit_windows"] == 1 and drv.stats["admit_window_reqs"] == 4
        assert drv.stats["admit_window_s"] < 0.25
        assert eng.stats["prefill_steps"] == 1
    finally:
        drv.stop()


def _own_driver(model_dir, **kw):
    m = build_model(model_dir, None, "fp32", "cpu")
    tok = load_tokenizer(model_dir, m.cfg.vocab_size)
    eng = LLMEngine(m, max_num_seqs=8, block_size=4, num_blocks=256, eos_token_id=None, **kw)
    return EngineDriver(eng), tok


@pytest.mark.parametrize("expecting", [True, False])
def test_admission_window_waits_longer_for_expected_resubmissions(model_dir, expecting):
    """Closed-loop clients behind the pub/sub hops re-submit spread over more than one quiet period: after 6 replies,
    6 arrivals in groups 2.5 windows apart, 12.5 windows in all (past batch_window_max), are still ONE prefill step:
    while fewer arrivals than recent replies came, the window tolerates a 4x gap and stays open up to
    resubmit_windows. Without the expectation (horizon 0) the same arrivals take several steps."""
    drv, tok = _own_driver(model_dir)
    drv.batch_window_s = 0.02
    drv.resubmit_horizon_s = 30.0 if expecting else 0.0
    drv.start()
    eng = drv.engine
    try:
        sp = SamplingParams(max_new_tokens=3, is_greedy=True)
        hs = [drv.submit(encode(tok, f"first {i}"), sp) for i in range(6)]
        assert all(h.wait(60) for h in hs)
        time.sleep(0.2)  # the engine is idle again
        before = eng.stats["prefill_steps"]
        hs = []
        for i in range(6):
            if i:
                time.sleep(0.05)
            hs.append(drv.submit(encode(tok, f"again {i}"), sp))
        assert all(h.wait(60) for h in hs)
        steps = eng.stats["prefill_steps"] - before
        assert steps == 1 if expecting else steps >= 2, (steps, list(drv.admit_log))
    finally:
        drv.stop()


def test_admission_holds_arrivals_while_the_engine_is_about_to_drain(model_dir):
    """Arrivals while every running sequence is within merge_steps tokens of its limit are held back and admitted
    with the next idle window (with the re-submissions of the finishing sequences) - unless the cap runs out. Far
    from the limit they are admitted at once. Driven by hand: no driver thread."""
    drv, tok = _own_driver(model_dir)
    eng = drv.engine
    drv.merge_steps = 3
    drv.batch_window_s, drv.batch_window_max = 0.01, 100000  # the hold cap cannot run out in this test
    eng.add_request(encode(tok, "running"), SamplingParams(max_new_tokens=3, is_greedy=True))
    eng.step()  # prefill: the sequence runs, 3 tokens or fewer left
    h = drv.submit(encode(tok, "arrives"), SamplingParams(max_new_tokens=3, is_greedy=True))
    msg = drv._collect(block=False)
    assert msg["new"] == [] and [it[1].rid for it in drv._held] == [h.rid] and drv.stats["admit_held"] == 1
    msg = drv._collect(block=False)  # still near the drain: still held, counted once
    assert msg["new"] == [] and len(drv._held) == 1 and drv.stats["admit_held"] == 1
    while eng.has_unfinished():
        eng.step()
    eng.pop_finished()
    msg = drv._collect(block=True)
    assert [r[0] for r in msg["new"]] == [h.rid] and not drv._held
    # far from the limit: admitted at once
    eng.add_request(encode(tok, "long"), SamplingParams(max_new_tokens=50, is_greedy=True))
    eng.step()
    h2 = drv.submit(encode(tok, "arrives 2"), SamplingParams(max_new_tokens=3, is_greedy=True))
    assert [r[0] for r in drv._collect(block=False)["new"]] == [h2.rid]
    # the cap: a hold never outlives batch_window_max windows from the first held arrival
    drv2, _ = _own_driver(model_dir)
    drv2.merge_steps, drv2.batch_window_s = 3, 0.001
    drv2.engine.add_request(encode(tok, "running"), SamplingParams(max_new_tokens=3, is_greedy=True))
    drv2.engine.step()
    h3 = drv2.submit(encode(tok, "arrives 3"), SamplingParams(max_new_tokens=3, is_greedy=True))
    drv2._held_t = time.perf_counter()
    drv2._held = [drv2.inbox.get_nowait()]
    time.sleep(0.05)
    assert [r[0] for r in drv2._collect(block=False)["new"]] == [h3.rid] and not drv2._held


def test_aio_server_stop_after_its_loop_ended(driver):
    """stop().wait() returns when the server's loop already ended (it used to schedule the stop onto the dead
    loop and wait forever)."""
    drv, tok, m = driver
    server = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
    server.loop.call_soon_threadsafe(server.loop.stop)  # the loop ends without a server stop
    server._thread.join(10)
    assert not server._thread.is_alive()
    t0 = time.perf_counter()
    assert server.stop(0).wait(5)
    assert time.perf_counter() - t0 < 5
    ok = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")  # the normal path still stops cleanly
    assert ok.stop(0).wait(30)


def test_aio_server_stop_completes_on_its_own_loop(driver):
    """Root cause of round 4's stuck stop (profiles/r4_serving): the server signals termination part-way through
    its own stop(), so a stop coroutine scheduled from outside raced the loop's exit and never finished. Now the
    loop's main task runs server.stop(grace) itself: with streams in flight, stop().wait() returns, the stop ran
    to the end (stop_completed), the streams end, pending servicer tasks are drained, the loop is closed and the
    port refuses new calls - five times in a row."""
    import threading

    drv, tok, m = driver
    for _ in range(5):
        server = serve(EngineServicer(drv, tok), port=0, host="127.0.0.1")
        ch = grpc.insecure_channel(f"127.0.0.1:{server.bound_port}")
        stub = Stub(ch)
        got, errs = [], []

        def stream():
            try:
                for t in stub.GenerateStream(GenerateRequest(prompt="hello world", max_new_tokens=400, is_greedy=True,
                                                             ignore_eos=True), timeout=60):
                    got.append(t)
            except grpc.RpcError as e:
                errs.append(e.code())
        th = threading.Thread(target=stream)
        th.start()
        t0 = time.perf_counter()
        while not got and time.perf_counter() - t0 < 30:
            time.sleep(0.01)
        assert got, "stream never started"
        assert server.stop(0.2).wait(30)
        assert server.stop_completed and server.loop.is_closed()
        th.join(30)
        assert not th.is_alive()
        with pytest.raises(grpc.RpcError):
            stub.Generate(GenerateRequest(prompt="x", max_new_tokens=1), timeout=5)
        ch.close()


@pytest.mark.parametrize("mode", [["--mode", "pubsub"], ["--mode", "pubsub", "--frontend-inproc"], ["--mode", "grpc"]])
def test_serving_bench_runs_on_cpu(mode):
    """bench/serving_bench.py end to end on a tiny model: client process, (for pub/sub) the front-end + broker
    process, consumer and engine; one JSON line whose requests were all answered."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench", "serving_bench.py"), "--model", "tiny-llama",
                        "--clients", "3", "--requests", "2", "--prompt-len", "12", "--gen-len", "4"] + mode,
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["requests"] == 6 and d["value"] > 0
    assert d["frontend"] == (None if "grpc" in mode else ("in-process" if "--frontend-inproc" in mode else "own process"))


def test_servicer_reports_an_expired_server_deadline_as_deadline_exceeded():
    """The driver holds a copy of the call's deadline; when that copy fires before the servicer's own wait, the
    call still ends DEADLINE_EXCEEDED (unary and streaming), never OK with a silently truncated output."""
    import asyncio
    import types

    from llmss_amd.serving.grpc_api import EngineServicer, GenerateRequest

    class Aborted(Exception):
        pass

    class Ctx:
        def time_remaining(self):
            return 30.0

        async def abort(self, code, msg):
            raise Aborted(code)

    class Drv:  # finishes every request at once as the driver's deadline check would: partial tokens, "deadline"
        def submit(self, ids, params, deadline_s=None, on_done=None, sink=None, sink_q=None):
            h = types.SimpleNamespace(rid=1, output_ids=[3, 4], finish_reason="deadline", error="deadline exceeded",
                                      metrics={}, done=threading.Event())
            h.done.set()
            if sink_q is not None:
                for t in (3, 4, None):
                    sink_q.put_nowait(t)
            if on_done is not None:
                on_done(h)
            return h

        def abort(self, rid):
            pass

    tok = types.SimpleNamespace(decode=lambda ids: "", convert_ids_to_tokens=lambda ids: [])
    sv = EngineServicer(Drv(), tok)
    req = GenerateRequest(prompt_token_ids=[1, 2], max_new_tokens=50, is_greedy=True)

    async def unary():
        await sv.Generate(req, Ctx())

    async def stream():
        async for _ in sv.GenerateStream(req, Ctx()):
            pass

    for f in (unary, stream):
        with pytest.raises(Aborted) as e:
            asyncio.run(f())
        assert e.value.args[0] == grpc.StatusCode.DEADLINE_EXCEEDED


@pytest.mark.parametrize("kind", ["memory", "resp"])
def test_broker_expire(kind):
    """EXPIRE as Redis: the key is gone after its TTL (lazily on access, and swept when nobody touches it again); a
    list that empties loses its TTL with it; EXPIRE on a missing key is 0."""
    srv = MiniRedisServer().start() if kind == "resp" else None
    b = RedisBroker(srv.host, srv.port) if srv else MemoryBroker()
    try:
        assert b.expire("none", 1) == 0
        b.lpush("a", "x")
        b.lpush("b", "y")
        b.lpush("c", "z")
        assert b.expire("a", 1) == 1 and b.expire("b", 1) == 1
        assert b.rpop("b") == "y"  # emptied: deleted, TTL gone with it
        b.lpush("b", "y2")
        time.sleep(1.3)
        assert b.llen("a") == 0 and b.lrange("a", 0, -1) == []  # expired
        assert b.lrange("b", 0, -1) == ["y2"] and b.llen("c") == 1  # no TTL / never had one
        b.lpush("d", "w")
        assert b.expire("d", 1) == 1
        time.sleep(1.3)
        b.llen("c")  # any command sweeps: "d" is dropped although nobody asks for it
        store = srv._lists if srv else b._lists
        assert "d" not in store and "a" not in store
        assert b.pipeline([("LPUSH", "e", "v"), ("EXPIRE", "e", 5)]) == [1, 1]
    finally:
        if srv:
            srv.stop()


def test_consumer_expires_replies_and_honours_request_deadlines(driver):
    """The pub/sub path bounds what an abandoned call costs: the request carries its caller's deadline (the engine
    stops generating then) and every reply list gets a TTL (a reply nobody pops is deleted by the broker)."""
    from llmss_amd.serving.broker import PQUEUE, reply_key

    drv, tok, m = driver
    b = MemoryBroker()
    consumer = Consumer(drv, tok, b, poll_timeout=0.05, durable=False, reply_ttl_s=3).start()
    try:
        b.lpush(PQUEUE, json.dumps({"prompt": "y", "prompt_token_ids": [4, 5], "max_new_tokens": 2, "is_greedy": True,
                                    "ignore_eos": True, "request_id": "gone"}))
        t0 = time.time()
        while b.llen(reply_key("gone")) == 0 and time.time() - t0 < 30:
            time.sleep(0.02)
        assert b.llen(reply_key("gone")) == 1  # answered, never popped ...
        b.lpush(PQUEUE, json.dumps({"prompt": "x", "prompt_token_ids": [1, 2, 3], "max_new_tokens": 100000,
                                    "is_greedy": True, "ignore_eos": True, "request_id": "late", "deadline_s": 0.0}))
        late = json.loads(b.brpop(reply_key("late"), timeout=60))
        assert late["finish_reason"] == "deadline" and late["output_tokens"] < 100000
        time.sleep(max(0.0, t0 + 4.0 - time.time()))
        assert b.llen(reply_key("gone")) == 0  # ... and expired
    finally:
        consumer.stop()
