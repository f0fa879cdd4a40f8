"""Front-end of the pub/sub path: FastAPI ``POST /generate`` (+ optional gRPC) -> broker.

Reference: producer_server.py:43-57 - ``async def generate`` pushes the request, then busy-spins
on ``LLEN/RPOP squeue`` with a *synchronous* Redis client inside the event loop (serialising all
requests and mixing up replies between concurrent clients, quirk Q11). Here every request gets a
``request_id`` and waits on its own reply key with a blocking pop run in a worker thread, so the
event loop keeps accepting requests and replies can never be swapped.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Optional

from fastapi import FastAPI, HTTPException
from fastapi.responses import PlainTextResponse

from .broker import PQUEUE, Broker, reply_key
from .protocol import Request, Response, new_request_id


def create_app(broker: Broker, timeout_s: float = 600.0) -> FastAPI:
    app = FastAPI(title="llmss_amd producer")
    stats = {"requests": 0, "completed": 0, "timeouts": 0, "latency_s_sum": 0.0}

    @app.post("/generate")
    async def generate(request: Request) -> Response:
        rid = request.request_id or new_request_id()
        # the consumer stops generating when this endpoint stops waiting for the reply
        wait_s = min(timeout_s, request.deadline_s) if request.deadline_s else timeout_s
        req = request.model_copy(update={"request_id": rid, "deadline_s": wait_s})
        t0 = time.perf_counter()
        stats["requests"] += 1
        await asyncio.to_thread(broker.lpush, PQUEUE, req.model_dump_json())
        msg: Optional[str] = await asyncio.to_thread(broker.brpop, reply_key(rid), wait_s)
        if msg is None:
            stats["timeouts"] += 1
            raise HTTPException(status_code=504, detail="generation timed out")
        stats["completed"] += 1
        stats["latency_s_sum"] += time.perf_counter() - t0
        d = json.loads(msg)
        return Response(**{k: d.get(k) for k in Response.model_fields if k in d})

    @app.get("/health")
    async def health():
        return {"status": "ok"}

    @app.get("/metrics", response_class=PlainTextResponse)
    async def metrics():
        lines = [f"llmss_producer_{k} {v}" for k, v in stats.items()]
        return "\n".join(lines) + "\n"

    return app
