"""Shared-memory control ring (csrc/ctrl.cpp): the serving driver's leader -> follower channel on one node.

CPU-only: one producer, several reader processes; fragmentation of messages larger than a quarter of the
ring, wrap-around with back-pressure (more bytes in flight than the ring holds), timeouts, orderly close,
and that the name is gone from /dev/shm once every reader attached.
"""
import hashlib
import multiprocessing as mp
import os
import uuid

import pytest

from llmss_amd import _native


def _name():
    return f"/llmss_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"


def _msgs(n):
    out = []
    for i in range(n):
        size = [0, 1, 7, 8, 100, 5000, 70000, 300000][i % 8]  # 70000 / 300000 > capacity / 4: fragmented
        out.append(bytes((i * 31 + j) & 255 for j in range(size)) if size < 6000 else os.urandom(size))
    return out


def _reader(name, idx, n, q):
    try:
        C = _native()
        r = C.CtrlRing(name, False, 0, 0, idx)
        digests = [hashlib.sha1(r.recv(30.0)).hexdigest() for _ in range(n)]
        try:
            r.recv(30.0)
            tail = "no-close"
        except RuntimeError as e:
            tail = "closed" if "closed" in str(e) else repr(e)
        q.put((idx, digests, tail))
    except Exception as e:  # noqa: BLE001
        q.put((idx, repr(e), ""))


def test_ring_many_readers_fragments_and_wraparound():
    C = _native()
    name = _name()
    nreaders, n = 3, 48
    ring = C.CtrlRing(name, True, 1 << 16, nreaders, 0)  # 64 KiB ring, ~3 MB of traffic
    assert ring.capacity == 1 << 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_reader, args=(name, i, n, q)) for i in range(nreaders)]
    for p in procs:
        p.start()
    try:
        assert ring.wait_attached(60.0)
        assert not os.path.exists("/dev/shm" + name)  # unlinked once everyone mapped it
        msgs = _msgs(n)
        for m in msgs:
            ring.send(m, 30.0)
        ring.close_producer()
        want = [hashlib.sha1(m).hexdigest() for m in msgs]
        for _ in range(nreaders):
            idx, got, tail = q.get(timeout=120)
            assert got == want, f"reader {idx}: {got if isinstance(got, str) else 'digest mismatch'}"
            assert tail == "closed"
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()


def test_ring_timeouts():
    C = _native()
    name = _name()
    ring = C.CtrlRing(name, True, 1 << 16, 1, 0)
    reader = C.CtrlRing(name, False, 0, 0, 0)
    assert ring.wait_attached(5.0)
    with pytest.raises(TimeoutError):
        reader.recv(0.05)  # nothing sent
    ring.send(b"x" * 10000, 1.0)
    assert reader.recv(1.0) == b"x" * 10000
    # a reader that stops reading: the producer fills the ring and then times out instead of overwriting
    with pytest.raises(TimeoutError):
        for _ in range(100):
            ring.send(b"y" * 8000, 0.05)
    got = reader.recv(1.0)
    assert got == b"y" * 8000


def test_ring_rejects_bad_args():
    C = _native()
    with pytest.raises(ValueError):
        C.CtrlRing("no_slash", True, 1 << 16, 1, 0)
    with pytest.raises(RuntimeError):
        C.CtrlRing(_name(), False, 0, 0, 0)  # nothing to attach to


def test_ring_close_drains_pending_records():
    """A record published right before close_producer() is still delivered; only then does recv raise."""
    C = _native()
    name = _name()
    ring = C.CtrlRing(name, True, 1 << 16, 1, 0)
    reader = C.CtrlRing(name, False, 0, 0, 0)
    assert ring.wait_attached(5.0)
    ring.send(b"stop-record", 1.0)
    ring.send(b"z" * 40000, 1.0)  # fragmented (> capacity / 4)
    ring.close_producer()
    assert reader.recv(1.0) == b"stop-record"
    assert reader.recv(1.0) == b"z" * 40000
    with pytest.raises(RuntimeError, match="closed"):
        reader.recv(1.0)


def test_ring_timeout_between_fragments_resumes_message():
    """A reader that times out in the middle of a fragmented message resumes it on the next recv() instead of
    returning the remaining fragments as a message of their own."""
    import threading

    C = _native()
    name = _name()
    ring = C.CtrlRing(name, True, 1 << 16, 2, 0)
    fast = C.CtrlRing(name, False, 0, 0, 0)
    slow = C.CtrlRing(name, False, 0, 0, 1)
    assert ring.wait_attached(5.0)
    first = b"a" * 40000
    big = os.urandom(60000)  # 4 fragments of ~16 KiB: only the first fits while `slow` holds `first`
    ring.send(first, 1.0)
    t = threading.Thread(target=ring.send, args=(big, 30.0))
    t.start()
    try:
        assert fast.recv(5.0) == first
        with pytest.raises(TimeoutError):
            fast.recv(0.2)  # one fragment of `big` is there, the rest waits for `slow`
        assert slow.recv(5.0) == first  # frees the ring: the producer finishes `big`
        assert fast.recv(5.0) == big
        assert slow.recv(5.0) == big
    finally:
        t.join(30)
