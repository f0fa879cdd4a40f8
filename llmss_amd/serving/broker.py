"""Request queue with Redis-list semantics (reference L5: external Redis lists ``pqueue`` /
``squeue``, producer_server.py:39-54, consumer_server.py:38-40,79-80,170-173).

* :class:`RedisBroker` - a minimal RESP2 client over a TCP socket (the ``redis`` package is not
  required); speaks to a real ``redis-server`` or to :class:`MiniRedisServer`.
* :class:`MemoryBroker` - thread-safe in-process lists (tests, single-process serving).
* :class:`MiniRedisServer` - a small single-threaded (asyncio) RESP server implementing the list commands the
  pub/sub path needs (LPUSH/RPUSH/LPOP/RPOP/LLEN/BRPOP/BLPOP/RPOPLPUSH/BRPOPLPUSH/LREM/LRANGE/DEL/PING), so the
  PoC runs where no ``redis-server`` is installed.

:meth:`Broker.pipeline` runs a list of commands in order; the RESP client writes them in one send and reads the
replies together (Redis pipelining), so a burst of replies or pops costs one round trip instead of one each.

Blocking pops (``brpop``) replace the reference's busy ``while True: if llen: rpop`` loops
(quirk Q11); replies are correlated by request id (``squeue:<id>``).
"""
from __future__ import annotations

import socket
import threading
import time
from collections import deque
from typing import Dict, List, Optional, Tuple

PQUEUE = "pqueue"
SQUEUE = "squeue"


def reply_key(request_id: Optional[str]) -> str:
    return f"{SQUEUE}:{request_id}" if request_id else SQUEUE


class Broker:
    def lpush(self, key: str, value: str) -> int:
        raise NotImplementedError

    def rpush(self, key: str, value: str) -> int:
        raise NotImplementedError

    def rpop(self, key: str) -> Optional[str]:
        raise NotImplementedError

    def lpop(self, key: str) -> Optional[str]:
        raise NotImplementedError

    def llen(self, key: str) -> int:
        raise NotImplementedError

    def brpop(self, key: str, timeout: float = 0) -> Optional[str]:
        """Blocking right-pop; ``timeout`` seconds (0 = forever). Returns the value or None."""
        raise NotImplementedError

    def brpoplpush(self, src: str, dst: str, timeout: float = 0) -> Optional[str]:
        """Pop the tail of ``src`` and push it onto the head of ``dst`` in one step (Redis BRPOPLPUSH): a
        consumer's in-flight request stays in its processing list until it is acknowledged with lrem."""
        raise NotImplementedError

    def rpoplpush(self, src: str, dst: str) -> Optional[str]:
        """Non-blocking RPOPLPUSH: None when ``src`` is empty."""
        raise NotImplementedError

    def lrem(self, key: str, count: int, value: str) -> int:
        raise NotImplementedError

    def expire(self, key: str, seconds: float) -> int:
        """Delete ``key`` after ``seconds`` unless it empties (and so disappears) first, as Redis EXPIRE: reply
        lists whose caller gave up are not kept forever. 1 if the key exists, else 0."""
        raise NotImplementedError

    def lrange(self, key: str, start: int, stop: int) -> List[str]:
        raise NotImplementedError

    def delete(self, key: str) -> int:
        raise NotImplementedError

    def pipeline(self, cmds: List[Tuple]) -> List:
        """Run ``cmds`` (tuples like ``("LPUSH", key, value)``) in order and return their replies; a command that
        fails yields its exception object in place of a reply, and the rest still run."""
        ops = {"LPUSH": self.lpush, "RPUSH": self.rpush, "RPOP": self.rpop, "LPOP": self.lpop, "LLEN": self.llen,
               "RPOPLPUSH": self.rpoplpush, "LREM": self.lrem, "DEL": self.delete, "EXPIRE": self.expire}
        out = []
        for c in cmds:
            try:
                out.append(ops[c[0].upper()](*c[1:]))
            except Exception as e:  # noqa: BLE001 - per-command result, like a RESP error reply
                out.append(e)
        return out

    def close(self):
        pass


# ------------------------------------------------------------------------------- in-memory
class MemoryBroker(Broker):
    """Thread-safe in-process lists. A blocking pop waits on its key's own condition, so a push wakes only the
    waiters of that key: with one shared condition every push woke every blocked pop (the pub/sub front-end's 64
    reply waiters: 64 x 64 wake-ups per batch of replies, each taking the interpreter lock - 60-75 ms for a
    GPT-2-XL cohort's re-submissions to get through, profiles/r6_pubsub). A list that empties is deleted, as in
    Redis, so one-shot reply keys leave nothing behind."""

    def __init__(self):
        self._lists: Dict[str, deque] = {}
        self._lock = threading.Lock()
        self._waiters: Dict[str, list] = {}  # key -> [Condition on self._lock, number of waiting threads]
        self._expiry: Dict[str, float] = {}  # key -> time.monotonic() deadline (EXPIRE)
        self._swept = 0.0

    def _live(self, key):  # lock held: the key's list, or None once it has expired (then deleted)
        self._sweep()
        t = self._expiry.get(key)
        if t is not None and time.monotonic() >= t:
            self._lists.pop(key, None)
            del self._expiry[key]
        return self._lists.get(key)

    def _sweep(self):  # lock held: drop expired keys nobody touches any more, at most once a second
        now = time.monotonic()
        if now - self._swept >= 1.0:
            self._swept = now
            for k in [k for k, t in self._expiry.items() if now >= t]:
                self._lists.pop(k, None)
                del self._expiry[k]

    def expire(self, key, seconds):
        with self._lock:
            self._sweep()
            if self._live(key) is None:
                return 0
            self._expiry[key] = time.monotonic() + float(seconds)
            return 1

    def _push(self, key, value, left):  # lock held
        q = self._live(key)
        if q is None:
            q = self._lists[key] = deque()
        if left:
            q.appendleft(value)
        else:
            q.append(value)
        w = self._waiters.get(key)
        if w is not None:
            w[0].notify()  # one element satisfies one pop
        return len(q)

    def _pop(self, key, right=True):  # lock held
        q = self._live(key)
        if not q:
            return None
        v = q.pop() if right else q.popleft()
        if not q:
            del self._lists[key]
            self._expiry.pop(key, None)
        return v

    def _wait(self, key, rem):  # lock held; False once the deadline has passed
        if rem is not None and rem <= 0:
            return False
        w = self._waiters.get(key)
        if w is None:
            w = self._waiters[key] = [threading.Condition(self._lock), 0]
        w[1] += 1
        try:
            w[0].wait(rem)
        finally:
            w[1] -= 1
            if w[1] == 0:
                del self._waiters[key]
        return True

    def _blocking(self, key, timeout, take):
        deadline = None if not timeout else time.monotonic() + timeout
        with self._lock:
            while True:
                v = take()
                if v is not None:
                    w = self._waiters.get(key)
                    if w is not None and self._lists.get(key):
                        w[0].notify()  # more elements left than this pop took: pass the wake-up on
                    return v
                if not self._wait(key, None if deadline is None else deadline - time.monotonic()):
                    return None

    def lpush(self, key, value):
        with self._lock:
            return self._push(key, value, True)

    def rpush(self, key, value):
        with self._lock:
            return self._push(key, value, False)

    def rpop(self, key):
        with self._lock:
            return self._pop(key)

    def lpop(self, key):
        with self._lock:
            return self._pop(key, right=False)

    def llen(self, key):
        with self._lock:
            return len(self._live(key) or ())

    def brpop(self, key, timeout=0):
        return self._blocking(key, timeout, lambda: self._pop(key))

    def blpop(self, key, timeout=0):
        return self._blocking(key, timeout, lambda: self._pop(key, right=False))

    def delete(self, key):
        with self._lock:
            self._expiry.pop(key, None)
            return 1 if self._lists.pop(key, None) is not None else 0

    def _move(self, src, dst):  # lock held
        v = self._pop(src)
        if v is not None:
            self._push(dst, v, True)
        return v

    def brpoplpush(self, src, dst, timeout=0):
        return self._blocking(src, timeout, lambda: self._move(src, dst))

    def rpoplpush(self, src, dst):
        with self._lock:
            return self._move(src, dst)

    def lrem(self, key, count, value):
        """Remove up to ``count`` occurrences of ``value`` (0 = all; < 0 = from the tail), like Redis."""
        with self._lock:
            q = self._live(key)
            if not q:
                return 0
            items = list(q)
            idx = [i for i, v in enumerate(items) if v == value]
            if count < 0:
                idx = idx[::-1][:-count]
            elif count > 0:
                idx = idx[:count]
            drop = set(idx)
            rest = deque(v for i, v in enumerate(items) if i not in drop)
            if rest:
                self._lists[key] = rest
            else:
                del self._lists[key]
                self._expiry.pop(key, None)
            return len(drop)

    def lrange(self, key, start, stop):
        with self._lock:
            items = list(self._live(key) or ())
        n = len(items)
        start = max(0, start + n if start < 0 else start)
        stop = stop + n if stop < 0 else stop
        return items[start:stop + 1]


# ------------------------------------------------------------------------------- RESP client
def _encode(*args) -> bytes:
    out = [b"*%d\r\n" % len(args)]
    for a in args:
        b = a if isinstance(a, bytes) else str(a).encode("utf-8")
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


class _Reader:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = b""

    def _fill(self):
        chunk = self.sock.recv(65536)
        if not chunk:
            raise ConnectionError("RESP connection closed")
        self.buf += chunk

    def line(self) -> bytes:
        while b"\r\n" not in self.buf:
            self._fill()
        ln, self.buf = self.buf.split(b"\r\n", 1)
        return ln

    def exact(self, n: int) -> bytes:
        while len(self.buf) < n + 2:
            self._fill()
        data, self.buf = self.buf[:n], self.buf[n + 2:]
        return data

    def value(self):
        ln = self.line()
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RuntimeError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self.exact(n).decode("utf-8")
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.value() for _ in range(n)]
        raise RuntimeError(f"bad RESP type {t!r}")


class RedisBroker(Broker):
    """Thread-safe (one connection per thread) minimal Redis client."""

    def __init__(self, host: str = "127.0.0.1", port: int = 6379, connect_timeout: float = 10.0):
        self.host, self.port, self.connect_timeout = host, int(port), connect_timeout
        self._local = threading.local()

    def _conn(self) -> Tuple[socket.socket, _Reader]:
        c = getattr(self._local, "conn", None)
        if c is None:
            s = socket.create_connection((self.host, self.port), timeout=self.connect_timeout)
            s.settimeout(None)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = (s, _Reader(s))
            self._local.conn = c
        return c

    def execute(self, *args):
        s, r = self._conn()
        try:
            s.sendall(_encode(*args))
            return r.value()
        except (ConnectionError, OSError):
            self._local.conn = None
            raise

    def ping(self):
        return self.execute("PING")

    def lpush(self, key, value):
        return self.execute("LPUSH", key, value)

    def rpush(self, key, value):
        return self.execute("RPUSH", key, value)

    def rpop(self, key):
        return self.execute("RPOP", key)

    def lpop(self, key):
        return self.execute("LPOP", key)

    def llen(self, key):
        return self.execute("LLEN", key)

    def brpop(self, key, timeout=0):
        r = self.execute("BRPOP", key, _fmt_timeout(timeout))
        return None if r is None else r[1]

    def blpop(self, key, timeout=0):
        r = self.execute("BLPOP", key, _fmt_timeout(timeout))
        return None if r is None else r[1]

    def delete(self, key):
        return self.execute("DEL", key)

    def brpoplpush(self, src, dst, timeout=0):
        return self.execute("BRPOPLPUSH", src, dst, _fmt_timeout(timeout))

    def rpoplpush(self, src, dst):
        return self.execute("RPOPLPUSH", src, dst)

    def pipeline(self, cmds):
        if not cmds:
            return []
        s, r = self._conn()
        try:
            s.sendall(b"".join(_encode(*c) for c in cmds))
            out = []
            for _ in cmds:
                try:
                    out.append(r.value())
                except RuntimeError as e:  # an error reply; the stream stays in sync
                    out.append(e)
            return out
        except (ConnectionError, OSError):
            self._local.conn = None
            raise

    def lrem(self, key, count, value):
        return self.execute("LREM", key, int(count), value)

    def lrange(self, key, start, stop):
        return self.execute("LRANGE", key, int(start), int(stop)) or []

    def expire(self, key, seconds):
        return self.execute("EXPIRE", key, int(max(1, round(float(seconds)))))

    def close(self):
        c = getattr(self._local, "conn", None)
        if c is not None:
            c[0].close()
            self._local.conn = None


class AsyncRedisClient:
    """asyncio RESP client for coroutine front-ends (:class:`~llmss_amd.serving.grpc_api.AioBrokerServicer`): the
    commands of every in-flight request run on the server's event loop, not in a thread each. A pool of
    connections, one per concurrently blocked command (a BRPOP holds its connection until its reply); a command
    that is cancelled or fails closes its connection, whose reply stream is then out of step."""

    def __init__(self, host: str = "127.0.0.1", port: int = 6379):
        self.host, self.port = host, int(port)
        self._free: list = []

    async def execute(self, *args):
        import asyncio

        conn = self._free.pop() if self._free else None
        if conn is None:
            conn = await asyncio.open_connection(self.host, self.port)
            conn[1].get_extra_info("socket").setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        rd, wr = conn
        ok = False
        try:
            wr.write(_encode(*args))
            out = await self._value(rd)
            ok = True
            return out
        finally:
            if ok:
                self._free.append(conn)
            else:
                wr.close()

    async def _value(self, rd):
        ln = (await rd.readuntil(b"\r\n"))[:-2]
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RuntimeError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else (await rd.readexactly(n + 2))[:-2].decode("utf-8")
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [await self._value(rd) for _ in range(n)]
        raise RuntimeError(f"bad RESP type {t!r}")

    async def lpush(self, key, value):
        return await self.execute("LPUSH", key, value)

    async def brpop(self, key, timeout=0):
        r = await self.execute("BRPOP", key, _fmt_timeout(timeout))
        return None if r is None else r[1]

    def close(self):
        for _, wr in self._free:
            wr.close()
        self._free.clear()


def _fmt_timeout(t: float) -> str:
    return str(int(t)) if float(t).is_integer() else f"{t:.3f}"


# ------------------------------------------------------------------------------- mini server
class MiniRedisServer:
    """RESP server for the list commands of the pub/sub path, on ONE asyncio event-loop thread as Redis itself
    runs: a connection is a coroutine, a blocked pop a future parked on its key, and a push hands its element to
    the oldest parked pop of that key directly. The thread-per-connection server it replaces spent most of a
    cohort's turnaround handing the interpreter lock between its 64+ connection threads and the front-end's
    handlers (bench/pubsub_rtt.py, profiles/r6_pubsub)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        import asyncio

        self._lists: Dict[str, deque] = {}
        self._waiters: Dict[str, deque] = {}  # key -> parked pops: (future, take) with take(key) -> value
        self._expiry: Dict[str, float] = {}  # key -> time.monotonic() deadline (EXPIRE)
        self._swept = 0.0
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._sock.bind((host, port))
        self._sock.listen(512)
        self.host, self.port = self._sock.getsockname()[:2]
        self.loop = asyncio.new_event_loop()
        self._thread = threading.Thread(target=self._run, daemon=True, name="mini-redis")
        self._server = None
        self._conns: set = set()

    # list store (event-loop thread only)
    def _live(self, key):  # the key's list, or None once it has expired (then deleted)
        t = self._expiry.get(key)
        if t is not None and time.monotonic() >= t:
            self._lists.pop(key, None)
            del self._expiry[key]
        return self._lists.get(key)

    def _sweep(self):  # expired keys nobody touches any more, at most once a second
        now = time.monotonic()
        if now - self._swept >= 1.0:
            self._swept = now
            for k in [k for k, t in self._expiry.items() if now >= t]:
                self._lists.pop(k, None)
                del self._expiry[k]

    def _push(self, key, value, left):
        q = self._live(key)
        if q is None:
            q = self._lists[key] = deque()
        q.appendleft(value) if left else q.append(value)
        n = len(q)
        self._serve_waiters(key)
        return n

    def _pop(self, key, right=True):
        q = self._live(key)
        if not q:
            return None
        v = q.pop() if right else q.popleft()
        if not q:
            del self._lists[key]
            self._expiry.pop(key, None)
        return v

    def _serve_waiters(self, key):
        ws = self._waiters.get(key)
        while ws and self._lists.get(key):
            fut, take = ws.popleft()
            if not fut.done():
                fut.set_result(take(key))
        if ws is not None and not ws and self._waiters.get(key) is ws:  # a nested serve (a move onto the same key)
            del self._waiters[key]                                         # may have removed it already

    async def _blocking(self, keys, timeout, take):
        import asyncio

        for k in keys:
            if self._live(k):
                return k, take(k)
        fut = self.loop.create_future()
        for k in keys:
            self._waiters.setdefault(k, deque()).append((fut, lambda key, k=k: (k, take(key))))
        try:
            return await (asyncio.wait_for(fut, timeout) if timeout > 0 else fut)
        except asyncio.TimeoutError:
            return None
        finally:
            for k in keys:  # drop this pop's parked entries (served, timed out or cancelled)
                ws = self._waiters.get(k)
                if ws is not None:
                    rest = deque(w for w in ws if w[0] is not fut)
                    if rest:
                        self._waiters[k] = rest
                    else:
                        self._waiters.pop(k, None)

    def _move(self, src, dst):
        v = self._pop(src)
        if v is not None:
            self._push(dst, v, True)
        return v

    def _lrem(self, key, count, value):
        q = self._live(key)
        if not q:
            return 0
        items = list(q)
        idx = [i for i, v in enumerate(items) if v == value]
        idx = idx[::-1][:-count] if count < 0 else (idx[:count] if count > 0 else idx)
        drop = set(idx)
        rest = deque(v for i, v in enumerate(items) if i not in drop)
        if rest:
            self._lists[key] = rest
        else:
            del self._lists[key]
            self._expiry.pop(key, None)
        return len(drop)

    def _lrange(self, key, start, stop):
        items = list(self._live(key) or ())
        n = len(items)
        start = max(0, start + n if start < 0 else start)
        stop = stop + n if stop < 0 else stop
        return items[start:stop + 1]

    async def _exec(self, cmd):
        if not isinstance(cmd, list) or not cmd:
            raise RuntimeError("ERR protocol")
        op = cmd[0].upper()
        a = cmd[1:]
        self._sweep()
        if op == "PING":
            return "PONG"
        if op in ("LPUSH", "RPUSH"):
            n = 0
            for v in a[1:]:
                n = self._push(a[0], v, op == "LPUSH")
            return n
        if op in ("RPOP", "LPOP"):
            return ("bulk", self._pop(a[0], op == "RPOP"))
        if op == "LLEN":
            return len(self._live(a[0]) or ())
        if op in ("BRPOP", "BLPOP"):
            r = await self._blocking(a[:-1], float(a[-1]), lambda k: self._pop(k, op == "BRPOP"))
            return ("array", None if r is None else [r[0], r[1]])
        if op == "BRPOPLPUSH":
            r = await self._blocking([a[0]], float(a[2]), lambda k: self._move(k, a[1]))
            return ("bulk", None if r is None else r[1])
        if op == "RPOPLPUSH":
            return ("bulk", self._move(a[0], a[1]))
        if op == "DEL":
            for k in a:
                self._expiry.pop(k, None)
            return sum(1 for k in a if self._lists.pop(k, None) is not None)
        if op == "EXPIRE":
            if self._live(a[0]) is None:
                return 0
            self._expiry[a[0]] = time.monotonic() + float(a[1])
            return 1
        if op == "LREM":
            return self._lrem(a[0], int(a[1]), a[2])
        if op == "LRANGE":
            return ("array", self._lrange(a[0], int(a[1]), int(a[2])))
        raise RuntimeError(f"ERR unknown command {op}")

    async def _command(self, rd):
        ln = (await rd.readuntil(b"\r\n"))[:-2]
        if ln[:1] != b"*":
            raise RuntimeError("ERR protocol")
        out = []
        for _ in range(int(ln[1:])):
            hd = (await rd.readuntil(b"\r\n"))[:-2]
            if hd[:1] != b"$":
                raise RuntimeError("ERR protocol")
            out.append((await rd.readexactly(int(hd[1:]) + 2))[:-2].decode("utf-8"))
        return out

    async def _client(self, rd, wr):
        import asyncio

        wr.get_extra_info("socket").setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        task = asyncio.current_task()
        self._conns.add(task)
        try:
            while True:
                try:
                    cmd = await self._command(rd)
                except (asyncio.IncompleteReadError, ConnectionError, RuntimeError):
                    return
                try:
                    resp = await self._exec(cmd)
                except Exception as e:  # noqa: BLE001 - an error reply; the connection stays in step
                    resp = RuntimeError(str(e))
                wr.write(self._reply(resp))  # the transport sends at once; drain() waits only past its high-water mark
                await wr.drain()
        except (ConnectionError, OSError):
            return
        finally:
            self._conns.discard(task)
            wr.close()

    @staticmethod
    def _reply(r) -> bytes:
        if isinstance(r, Exception):
            return b"-%s\r\n" % str(r).encode()
        if isinstance(r, str):
            return b"+%s\r\n" % r.encode()
        if isinstance(r, int):
            return b":%d\r\n" % r
        kind, v = r
        if kind == "bulk":
            if v is None:
                return b"$-1\r\n"
            b = v.encode("utf-8")
            return b"$%d\r\n%s\r\n" % (len(b), b)
        if v is None:
            return b"*-1\r\n"
        return b"".join([b"*%d\r\n" % len(v)] + [MiniRedisServer._reply(("bulk", x)) for x in v])

    def _run(self):
        import asyncio

        asyncio.set_event_loop(self.loop)

        async def main():
            self._server = await asyncio.start_server(self._client, sock=self._sock)

        self.loop.run_until_complete(main())
        self.loop.run_forever()
        for t in list(self._conns):  # stop(): end the connection coroutines, then close the loop
            t.cancel()
        if self._conns:
            self.loop.run_until_complete(asyncio.gather(*self._conns, return_exceptions=True))
        self.loop.close()

    def start(self):
        self._thread.start()
        return self

    def stop(self):
        def _close():
            if self._server is not None:
                self._server.close()
            self.loop.stop()

        if self._thread.is_alive():
            self.loop.call_soon_threadsafe(_close)
            self._thread.join(10)
        else:
            self._sock.close()


def make_broker(host: Optional[str], port: Optional[int]) -> Broker:
    if host in (None, "", "memory"):
        return MemoryBroker()
    return RedisBroker(host, int(port))
