"""Back-end of the pub/sub path: a tensor-parallel consumer group (one rank per GPU).

Reference: consumer_server.py - rank 0 ``RPOP pqueue`` when ``LLEN`` > 0, ``batch_size = 1``, a
spinning ``broadcast_object_list`` every idle iteration, one request decoded to completion before
the next is popped, reply ``LPUSH squeue``; a consumer that dies loses the request it popped
(``consumer_server.py:79-80``).

Here rank 0 runs an intake thread that blocks on ``BRPOPLPUSH pqueue -> pqueue:processing:<id>`` and
submits every request to the :class:`EngineDriver` immediately, so concurrent requests share
continuous-batching decode steps; each completion is pushed to ``squeue:<request_id>`` (or plain
``squeue`` when the request came from a reference producer without an id) and only then removed
from the processing list (``LREM``). A consumer restarted under the same ``consumer_id`` first moves
whatever its previous incarnation left in that list back onto ``pqueue`` - a crash no longer loses
in-flight requests. Streaming requests (``"stream": true``) get one message per engine step with
that step's tokens, then the final message. Replies are written by a publisher thread, so the
engine loop never waits on the broker. All ranks run the driver loop; followers block on the CPU
control group between bursts of work.

Bursts cost one broker round trip, not one per request: the publisher sends everything it drained (replies,
streamed tokens, acknowledgements) as one pipeline, and after each blocking pop the intake takes whatever else is
queued with one pipeline of non-blocking pops (``intake_batch``), so requests that arrive together start in the
same engine step. Measured on the closed-loop serving bench: profiles/r5_pubsub.
"""
from __future__ import annotations

import collections
import json
import queue
import threading
from typing import Optional

from ..utils.logging import get_logger
from ..utils.tokenizer import encode
from .broker import PQUEUE, Broker, reply_key
from .driver import EngineDriver, Handle
from .protocol import dump_response, parse_request, to_sampling

log = get_logger(__name__)


def processing_key(consumer_id: str) -> str:
    return f"{PQUEUE}:processing:{consumer_id}"


class Consumer:
    def __init__(self, driver: EngineDriver, tokenizer, broker: Optional[Broker] = None, poll_timeout: float = 1.0,
                 consumer_id: str = "0", durable: bool = True, intake_batch: int = 32, reply_ttl_s: float = 300.0):
        self.driver = driver
        self.tok = tokenizer
        self.broker = broker
        self.poll_timeout = poll_timeout
        self.consumer_id = str(consumer_id)
        self.durable = durable
        self.intake_batch = max(1, int(intake_batch))
        # every reply list gets this TTL (EXPIRE): the reply of a caller that gave up (deadline, cancelled call,
        # front-end restart) is deleted by the broker instead of being kept forever
        self.reply_ttl_s = reply_ttl_s
        self._stop = threading.Event()
        self._out: "queue.Queue" = queue.Queue()
        self.served = 0
        self.requeued = 0
        # durable mode: raw requests submitted and not yet acknowledged (LREM sent successfully), to tell which
        # processing-list entries a failed batch pop left behind (_resync_processing)
        self._inflight: "collections.Counter[str]" = collections.Counter()
        self._inflight_mu = threading.Lock()

    # ------------------------------------------------------------------ publisher thread
    def _publish_loop(self):
        """Drain everything queued, merge each streaming request's tokens into one message per drain (order
        kept per request: its pending tokens go out before its final reply), publish."""
        while True:
            batch = [self._out.get()]
            while True:
                try:
                    batch.append(self._out.get_nowait())
                except queue.Empty:
                    break
            pending = {}  # id(req) -> (req, tokens)
            cmds = []  # this drain's broker writes, sent as one pipeline
            pk = processing_key(self.consumer_id)

            def flush(key=None):
                for k in ([key] if key is not None else list(pending)):
                    if k in pending:
                        req, toks = pending.pop(k)
                        cmds.append(("LPUSH", reply_key(req.request_id),
                                     json.dumps({"token_ids": toks, "text": self.tok.decode(toks)})))
            stop = False
            for item in batch:
                if item is None:
                    stop = True
                    break
                try:
                    kind = item[0]
                    if kind == "tokens":
                        _, req, toks = item
                        pending.setdefault(id(req), (req, []))[1].extend(toks)
                    elif kind == "done":
                        _, req, h, raw = item
                        flush(id(req))
                        cmds.append(("LPUSH", reply_key(req.request_id), self._reply(req, h)))
                        if raw is not None and self.durable:
                            cmds.append(("LREM", pk, 1, raw))  # acknowledged
                    elif kind == "error":
                        _, rid, err, raw = item
                        cmds.append(("LPUSH", reply_key(rid),
                                     json.dumps({"prompt": "", "continuation": "", "error": err})))
                        if raw is not None and self.durable:
                            cmds.append(("LREM", pk, 1, raw))
                except Exception:  # noqa: BLE001 - one bad completion must not kill the publisher
                    log.exception("consumer publish: could not format a reply")
            try:
                flush()
                if self.reply_ttl_s:
                    keys = dict.fromkeys(c[1] for c in cmds if c[0] == "LPUSH")  # reply lists, in order, once each
                    cmds += [("EXPIRE", k, int(max(1, round(self.reply_ttl_s)))) for k in keys]
                for r in self.broker.pipeline(cmds):
                    if isinstance(r, Exception):
                        log.error("consumer publish: broker error %s", r)
                # acknowledged: these requests no longer count as in flight (an ack that failed keeps its entry in
                # the processing list and in flight - a resync then does not serve it twice)
                acked = [c[3] for c in cmds if c[0] == "LREM"]
                if acked:
                    with self._inflight_mu:
                        self._inflight.subtract(acked)
                        self._inflight += collections.Counter()  # drop counts <= 0
            except Exception:  # noqa: BLE001 - a broker hiccup must not kill the publisher
                log.exception("consumer publish failed")
            if stop:
                return

    def _reply(self, req, h: Handle) -> str:
        m = h.metrics or {}
        resp = {"prompt": req.prompt, "continuation": self.tok.decode(h.output_ids)}
        if req.request_id:
            resp.update(request_id=req.request_id, output_tokens=len(h.output_ids), token_ids=list(h.output_ids),
                        finish_reason=h.finish_reason, ttft_s=m.get("ttft_s"), e2e_s=m.get("e2e_s"))
            if req.stream:
                resp.update(finished=True, text="")
        if h.finish_reason == "error":
            resp["error"] = h.error or "engine failure"
        self.served += 1
        return dump_response(resp)

    # ------------------------------------------------------------------ intake
    def recover(self) -> int:
        """Put back on pqueue what a previous consumer with this id left unacknowledged (it crashed or was
        killed mid-request). RPUSH: the recovered requests are popped next (consumers pop the tail)."""
        if not self.durable:
            return 0
        key = processing_key(self.consumer_id)
        n = 0
        for raw in reversed(self.broker.lrange(key, 0, -1)):  # oldest (tail) first back to the pop end
            self.broker.rpush(PQUEUE, raw)
            n += 1
        self.broker.delete(key)
        if n:
            log.warning("consumer %s: re-queued %d unacknowledged request(s)", self.consumer_id, n)
        self.requeued += n
        return n

    def intake_loop(self):
        """Rank 0: broker -> engine (non-spinning blocking pop, then the rest of the queue in one pipeline)."""
        pk = processing_key(self.consumer_id)
        backoff = 0.05
        while not self._stop.is_set():
            try:
                if self.durable:
                    msg = self.broker.brpoplpush(PQUEUE, pk, timeout=self.poll_timeout)
                else:
                    msg = self.broker.brpop(PQUEUE, timeout=self.poll_timeout)
            except (ConnectionError, OSError) as e:  # broker restarting / gone: reconnect on the next pop
                if self._stop.is_set():
                    return
                log.warning("consumer intake: broker unreachable (%s); retrying in %.2f s", e, backoff)
                self._stop.wait(backoff)
                backoff = min(2 * backoff, 2.0)
                continue
            backoff = 0.05
            if msg is None:
                continue
            msgs = [msg]
            if self.intake_batch > 1:
                pop = ("RPOPLPUSH", PQUEUE, pk) if self.durable else ("RPOP", PQUEUE)
                try:
                    more = self.broker.pipeline([pop] * (self.intake_batch - 1))
                except Exception:  # noqa: BLE001 - the popped request is still served
                    # the server may have run some of the pops before the connection dropped. Durable mode: those
                    # requests sit in this consumer's processing list - resync below picks them up. Non-durable
                    # mode: they are lost, as the reference's RPOP loses a request whose consumer dies
                    # (consumer_server.py:79-80); the connection drop fails every other broker call too.
                    log.exception("consumer intake: batch pop failed")
                    more = None
                if more is not None:
                    msgs += [m for m in more if isinstance(m, str)]
                elif self.durable:
                    for m in msgs:
                        self._submit(m)
                    msgs = self._resync_processing()
            for m in msgs:
                self._submit(m)

    def _resync_processing(self) -> list:
        """Durable mode, after a batch pop failed part-way: the entries of this consumer's processing list that are
        not in flight (popped by commands whose replies were lost). Returns them for submission."""
        try:
            listed = collections.Counter(self.broker.lrange(processing_key(self.consumer_id), 0, -1))
        except Exception:  # noqa: BLE001 - still unreachable: the next start's recover() re-queues them
            log.exception("consumer intake: processing-list resync failed")
            return []
        with self._inflight_mu:
            missing = listed - self._inflight
        out = [raw for raw, n in missing.items() for _ in range(n)]
        if out:
            log.warning("consumer %s: %d request(s) popped by a failed batch pop resubmitted", self.consumer_id,
                        len(out))
        return out

    def _submit(self, msg: str):
        raw = msg if self.durable else None
        if raw is not None:
            with self._inflight_mu:
                self._inflight[raw] += 1
        try:
            req = parse_request(msg)
            params = to_sampling(req)
        except Exception as e:  # noqa: BLE001  malformed request -> error reply, keep serving
            log.warning("bad request %r: %s", msg[:200], e)
            try:
                rid = json.loads(msg).get("request_id")
            except Exception:  # noqa: BLE001
                rid = None
            self._out.put(("error", rid, str(e), raw))
            return
        ids = list(req.prompt_token_ids) if req.prompt_token_ids else encode(self.tok, req.prompt)
        on_token = None
        if req.stream and req.request_id:
            def on_token(h, t, req=req):
                self._out.put(("tokens", req, [int(t)]))
        self.driver.submit(ids, params, on_done=lambda h, req=req, raw=raw: self._out.put(("done", req, h, raw)),
                           on_token=on_token, deadline_s=req.deadline_s)

    def start(self):
        if self.driver.leader:
            self.recover()
            self._pub = threading.Thread(target=self._publish_loop, daemon=True, name="broker-publish")
            self._pub.start()
            self._intake = threading.Thread(target=self.intake_loop, daemon=True, name="broker-intake")
            self._intake.start()
        return self

    def stop(self):
        self._stop.set()
        if self.driver.leader:
            self._out.put(None)
