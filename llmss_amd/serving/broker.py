"""Request queue with Redis-list semantics (reference L5: external Redis lists ``pqueue`` /
``squeue``, producer_server.py:39-54, consumer_server.py:38-40,79-80,170-173).

* :class:`RedisBroker` - a minimal RESP2 client over a TCP socket (the ``redis`` package is not
  required); speaks to a real ``redis-server`` or to :class:`MiniRedisServer`.
* :class:`MemoryBroker` - thread-safe in-process lists (tests, single-process serving).
* :class:`MiniRedisServer` - a small threaded RESP server implementing the list commands the
  pub/sub path needs (LPUSH/RPUSH/LPOP/RPOP/LLEN/BRPOP/BLPOP/RPOPLPUSH/BRPOPLPUSH/LREM/LRANGE/DEL/PING), so the
  PoC runs where no ``redis-server`` is installed.

:meth:`Broker.pipeline` runs a list of commands in order; the RESP client writes them in one send and reads the
replies together (Redis pipelining), so a burst of replies or pops costs one round trip instead of one each.

Blocking pops (``brpop``) replace the reference's busy ``while True: if llen: rpop`` loops
(quirk Q11); replies are correlated by request id (``squeue:<id>``).
"""
from __future__ import annotations

import socket
import socketserver
import threading
import time
from collections import defaultdict, deque
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

    def lrange(self, key: str, start: int, stop: int) -> List[str]:
        raise NotImplementedError

    def delete(self, key: str) -> int:
        raise NotImplementedError

    def pipeline(self, cmds: List[Tuple]) -> List:
        """Run ``cmds`` (tuples like ``("LPUSH", key, value)``) in order and return their replies; a command that
        fails yields its exception object in place of a reply, and the rest still run."""
        ops = {"LPUSH": self.lpush, "RPUSH": self.rpush, "RPOP": self.rpop, "LPOP": self.lpop, "LLEN": self.llen,
               "RPOPLPUSH": self.rpoplpush, "LREM": self.lrem, "DEL": self.delete}
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
    def __init__(self):
        self._lists: Dict[str, deque] = defaultdict(deque)
        self._cv = threading.Condition()

    def lpush(self, key, value):
        with self._cv:
            self._lists[key].appendleft(value)
            self._cv.notify_all()
            return len(self._lists[key])

    def rpush(self, key, value):
        with self._cv:
            self._lists[key].append(value)
            self._cv.notify_all()
            return len(self._lists[key])

    def rpop(self, key):
        with self._cv:
            q = self._lists.get(key)
            return q.pop() if q else None

    def lpop(self, key):
        with self._cv:
            q = self._lists.get(key)
            return q.popleft() if q else None

    def llen(self, key):
        with self._cv:
            return len(self._lists.get(key, ()))

    def brpop(self, key, timeout=0):
        deadline = None if not timeout else time.monotonic() + timeout
        with self._cv:
            while True:
                q = self._lists.get(key)
                if q:
                    return q.pop()
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return None
                self._cv.wait(rem)

    def blpop(self, key, timeout=0):
        deadline = None if not timeout else time.monotonic() + timeout
        with self._cv:
            while True:
                q = self._lists.get(key)
                if q:
                    return q.popleft()
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return None
                self._cv.wait(rem)

    def delete(self, key):
        with self._cv:
            return 1 if self._lists.pop(key, None) is not None else 0

    def brpoplpush(self, src, dst, timeout=0):
        deadline = None if not timeout else time.monotonic() + timeout
        with self._cv:
            while True:
                q = self._lists.get(src)
                if q:
                    v = q.pop()
                    self._lists[dst].appendleft(v)
                    self._cv.notify_all()
                    return v
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return None
                self._cv.wait(rem)

    def rpoplpush(self, src, dst):
        with self._cv:
            q = self._lists.get(src)
            if not q:
                return None
            v = q.pop()
            self._lists[dst].appendleft(v)
            self._cv.notify_all()
            return v

    def lrem(self, key, count, value):
        """Remove up to ``count`` occurrences of ``value`` (0 = all; < 0 = from the tail), like Redis."""
        with self._cv:
            q = self._lists.get(key)
            if not q:
                return 0
            items = list(q)
            idx = [i for i, v in enumerate(items) if v == value]
            if count < 0:
                idx = idx[::-1][:-count]
            elif count > 0:
                idx = idx[:count]
            drop = set(idx)
            self._lists[key] = deque(v for i, v in enumerate(items) if i not in drop)
            return len(drop)

    def lrange(self, key, start, stop):
        with self._cv:
            items = list(self._lists.get(key, ()))
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

    def close(self):
        c = getattr(self._local, "conn", None)
        if c is not None:
            c[0].close()
            self._local.conn = None


def _fmt_timeout(t: float) -> str:
    return str(int(t)) if float(t).is_integer() else f"{t:.3f}"


# ------------------------------------------------------------------------------- mini server
class MiniRedisServer:
    """Threaded RESP server over a :class:`MemoryBroker` (subset of Redis list commands)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.store = MemoryBroker()
        store = self.store

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                sock = self.request
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                rd = _Reader(sock)
                while True:
                    try:
                        cmd = rd.value()
                    except (ConnectionError, OSError):
                        return
                    try:
                        resp = MiniRedisServer._dispatch(store, cmd)
                    except Exception as e:  # noqa: BLE001
                        resp = RuntimeError(str(e))
                    try:
                        sock.sendall(MiniRedisServer._reply(resp))
                    except OSError:
                        return

        class Server(socketserver.ThreadingMixIn, socketserver.TCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self.server = Server((host, port), Handler)
        self.host, self.port = self.server.server_address
        self._thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    @staticmethod
    def _dispatch(store: MemoryBroker, cmd: List[str]):
        if not isinstance(cmd, list) or not cmd:
            raise RuntimeError("ERR protocol")
        op = cmd[0].upper()
        a = cmd[1:]
        if op == "PING":
            return "PONG"
        if op == "LPUSH":
            n = 0
            for v in a[1:]:
                n = store.lpush(a[0], v)
            return n
        if op == "RPUSH":
            n = 0
            for v in a[1:]:
                n = store.rpush(a[0], v)
            return n
        if op == "RPOP":
            return ("bulk", store.rpop(a[0]))
        if op == "LPOP":
            return ("bulk", store.lpop(a[0]))
        if op == "LLEN":
            return store.llen(a[0])
        if op in ("BRPOP", "BLPOP"):
            keys, t = a[:-1], float(a[-1])
            fn = store.brpop if op == "BRPOP" else store.blpop
            deadline = None if t == 0 else time.monotonic() + t
            while True:  # poll the keys in order (subset of Redis semantics, fine for one key)
                for k in keys:
                    v = (store.rpop if op == "BRPOP" else store.lpop)(k)
                    if v is not None:
                        return ("array", [k, v])
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return ("array", None)
                v = fn(keys[0], min(rem, 0.05) if rem is not None else 0.05)
                if v is not None:
                    return ("array", [keys[0], v])
        if op == "DEL":
            return sum(store.delete(k) for k in a)
        if op == "BRPOPLPUSH":
            t = float(a[2])
            deadline = None if t == 0 else time.monotonic() + t
            while True:  # bounded waits so a stopping server is not held by an idle client
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    return ("bulk", None)
                v = store.brpoplpush(a[0], a[1], min(rem, 0.05) if rem is not None else 0.05)
                if v is not None:
                    return ("bulk", v)
        if op == "RPOPLPUSH":
            return ("bulk", store.rpoplpush(a[0], a[1]))
        if op == "LREM":
            return store.lrem(a[0], int(a[1]), a[2])
        if op == "LRANGE":
            return ("array", store.lrange(a[0], int(a[1]), int(a[2])))
        raise RuntimeError(f"ERR unknown command {op}")

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

    def start(self):
        self._thread.start()
        return self

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


def make_broker(host: Optional[str], port: Optional[int]) -> Broker:
    if host in (None, "", "memory"):
        return MemoryBroker()
    return RedisBroker(host, int(port))
