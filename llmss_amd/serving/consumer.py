"""Back-end of the pub/sub path: a tensor-parallel consumer group (one rank per GPU).

Reference: consumer_server.py - rank 0 ``RPOP pqueue`` when ``LLEN`` > 0, ``batch_size = 1``, a
spinning ``broadcast_object_list`` every idle iteration, one request decoded to completion before
the next is popped, reply ``LPUSH squeue``.

Here rank 0 runs an intake thread that blocks on ``BRPOP pqueue`` and submits every request to the
:class:`EngineDriver` immediately, so concurrent requests share continuous-batching decode steps;
each completion is pushed to ``squeue:<request_id>`` (or plain ``squeue`` when the request came
from a reference producer without an id). All ranks run the driver loop; followers block on the
CPU control group between bursts of work.
"""
from __future__ import annotations

import json
import threading
from typing import Optional

from ..utils.logging import get_logger
from ..utils.tokenizer import encode
from .broker import PQUEUE, Broker, reply_key
from .driver import EngineDriver, Handle
from .protocol import dump_response, parse_request, to_sampling

log = get_logger(__name__)


class Consumer:
    def __init__(self, driver: EngineDriver, tokenizer, broker: Optional[Broker] = None, poll_timeout: float = 1.0):
        self.driver = driver
        self.tok = tokenizer
        self.broker = broker
        self.poll_timeout = poll_timeout
        self._stop = threading.Event()
        self.served = 0

    def _reply(self, req, h: Handle):
        m = h.metrics or {}
        resp = {"prompt": req.prompt, "continuation": self.tok.decode(h.output_ids)}
        if req.request_id:
            resp.update(request_id=req.request_id, output_tokens=len(h.output_ids), token_ids=list(h.output_ids),
                        finish_reason=h.finish_reason,
                        ttft_s=m.get("ttft_s"), e2e_s=m.get("e2e_s"))
        self.broker.lpush(reply_key(req.request_id), dump_response(resp))
        self.served += 1

    def intake_loop(self):
        """Rank 0: broker -> engine (non-spinning blocking pop)."""
        while not self._stop.is_set():
            msg = self.broker.brpop(PQUEUE, timeout=self.poll_timeout)
            if msg is None:
                continue
            try:
                req = parse_request(msg)
                params = to_sampling(req)
            except Exception as e:  # noqa: BLE001  malformed request -> error reply, keep serving
                log.warning("bad request %r: %s", msg[:200], e)
                try:
                    rid = json.loads(msg).get("request_id")
                except Exception:  # noqa: BLE001
                    rid = None
                self.broker.lpush(reply_key(rid), json.dumps({"prompt": "", "continuation": "", "error": str(e)}))
                continue
            ids = encode(self.tok, req.prompt)
            self.driver.submit(ids, params, on_done=lambda h, req=req: self._reply(req, h))

    def start(self):
        if self.driver.leader:
            self._intake = threading.Thread(target=self.intake_loop, daemon=True, name="broker-intake")
            self._intake.start()
        return self

    def stop(self):
        self._stop.set()
