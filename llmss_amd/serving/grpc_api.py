"""gRPC ``llmss.Generate`` service (``proto/generate.proto``). The reference advertises gRPC in its
README tagline (README.md:2) but ships none; this is new API surface (BASELINE north star).

``grpc_tools``/``protoc`` are not available, so the message classes are built at import time from
a ``FileDescriptorProto`` that mirrors ``proto/generate.proto`` field for field, and the service
is registered with generic method handlers. Any standard gRPC client generated from the .proto
file interoperates (same package, service, method and field numbers).

Two servicers:
* :class:`EngineServicer` - in-process on the TP leader, feeding :class:`EngineDriver` directly
  (lowest latency; config "GPT-2-XL TP=1 served over gRPC"). Its handlers are coroutines served by a
  ``grpc.aio`` server on an event-loop thread of its own: a request holds a future completed by the
  driver's ``on_done`` callback, not a pool thread parked in ``Handle.wait`` - with one thread per
  in-flight request, a 64-request burst took ~20 ms to dispatch and the 64 replies ~15 ms to go out
  (Python per-call overhead under one GIL), about half of that on the event loop.
* :class:`BrokerServicer` - a front-end that enqueues to the pub/sub broker and waits for the
  correlated reply (config "pub/sub producer/consumer under concurrent gRPC clients");
  :class:`AioBrokerServicer` is its coroutine form on a RESP broker (what the deployed front-ends run).
"""
from __future__ import annotations

import asyncio
import inspect
import json
import logging
import threading
import time
from concurrent import futures
from typing import Optional

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

log = logging.getLogger(__name__)

_F = descriptor_pb2.FieldDescriptorProto


def _build_pool():
    fd = descriptor_pb2.FileDescriptorProto(name="llmss/generate.proto", package="llmss", syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, (fname, ftype, rep) in enumerate(fields, 1):
            m.field.add(name=fname, number=num, type=ftype,
                        label=_F.LABEL_REPEATED if rep else _F.LABEL_OPTIONAL)

    S, I32, I64, B, FL = _F.TYPE_STRING, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_BOOL, _F.TYPE_FLOAT
    msg("GenerateRequest", [("prompt", S, 0), ("max_new_tokens", I32, 0), ("is_greedy", B, 0), ("temperature", FL, 0),
                            ("top_p", FL, 0), ("top_k", I32, 0), ("request_id", S, 0), ("seed", I64, 0),
                            ("prompt_token_ids", I32, 1), ("ignore_eos", B, 0)])
    msg("GenerateResponse", [("prompt", S, 0), ("continuation", S, 0), ("request_id", S, 0), ("token_ids", I32, 1),
                             ("finish_reason", S, 0), ("ttft_s", FL, 0), ("e2e_s", FL, 0)])
    msg("Token", [("token_id", I32, 0), ("text", S, 0), ("finished", B, 0), ("finish_reason", S, 0)])
    msg("StatsRequest", [])
    msg("StatsResponse", [("json", S, 0)])
    svc = fd.service.add(name="Generate")
    svc.method.add(name="Generate", input_type=".llmss.GenerateRequest", output_type=".llmss.GenerateResponse")
    svc.method.add(name="GenerateStream", input_type=".llmss.GenerateRequest", output_type=".llmss.Token",
                   server_streaming=True)
    svc.method.add(name="Stats", input_type=".llmss.StatsRequest", output_type=".llmss.StatsResponse")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return pool


_POOL = _build_pool()
GenerateRequest = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("llmss.GenerateRequest"))
GenerateResponse = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("llmss.GenerateResponse"))
Token = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("llmss.Token"))
StatsRequest = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("llmss.StatsRequest"))
StatsResponse = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("llmss.StatsResponse"))

SERVICE = "llmss.Generate"


def _params(req):
    from ..engine.sampling import SamplingParams

    # proto3 scalars default to 0: 0 means "reference default" for max_new_tokens/temperature/top_p
    # (0 is invalid for them) and "disabled" for top_k (as in the reference CLI, generate.py:30).
    return SamplingParams(max_new_tokens=req.max_new_tokens or 20, is_greedy=req.is_greedy,
                          temperature=req.temperature or 1.0, top_p=req.top_p or 0.95, top_k=req.top_k,
                          seed=req.seed or None, ignore_eos=req.ignore_eos).validate()


def add_servicer(server: grpc.Server, servicer) -> None:
    handlers = {
        "Generate": grpc.unary_unary_rpc_method_handler(
            servicer.Generate, request_deserializer=GenerateRequest.FromString,
            response_serializer=GenerateResponse.SerializeToString),
        "GenerateStream": grpc.unary_stream_rpc_method_handler(
            servicer.GenerateStream, request_deserializer=GenerateRequest.FromString,
            response_serializer=Token.SerializeToString),
        "Stats": grpc.unary_unary_rpc_method_handler(
            servicer.Stats, request_deserializer=StatsRequest.FromString,
            response_serializer=StatsResponse.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))


def serve(servicer, port: int = 50051, host: str = "0.0.0.0", max_workers: int = 64):
    """Start a gRPC server for ``servicer``: a ``grpc.aio`` server on its own event-loop thread when the
    servicer's handlers are coroutines (:class:`EngineServicer`), else a thread-pool server (blocking
    handlers, :class:`BrokerServicer`). Either object has ``bound_port`` and ``stop(grace).wait()``."""
    if inspect.iscoroutinefunction(getattr(servicer, "Generate", None)):
        return AioServer(servicer, port, host)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_receive_message_length", 64 << 20)])
    add_servicer(server, servicer)
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    server.bound_port = bound
    return server


class AioServer:
    """``grpc.aio`` server running on a dedicated event-loop thread (the engine driver keeps its own thread).

    The loop's one task, ``main``, owns the server's whole life: it starts the server, waits for either a stop
    request or the server terminating on its own, runs ``server.stop(grace)`` ITSELF, and only then returns -
    after which every task still pending on the loop (servicer coroutines of cancelled calls) is cancelled and
    drained and the loop is closed. Root cause of round 4's "loop ended early" (profiles/r4_serving): ``stop()``
    used to schedule ``server.stop()`` onto the loop from another thread while ``main`` awaited
    ``wait_for_termination()``. The server signals termination part-way through its own ``stop()``, so ``main``
    returned, ``run_until_complete`` stopped the loop, and the scheduled stop coroutine was left unfinished
    forever: the thread was gone and the caller's future never resolved (the stack dump's picture). Nothing
    ended early; the stop raced the loop's own exit (tests/test_serving.py)."""

    def __init__(self, servicer, port: int, host: str):
        self.loop = asyncio.new_event_loop()
        self.bound_port = None
        self._server = None
        self._err: Optional[BaseException] = None
        self._ready = threading.Event()
        self._stop_ev: Optional[asyncio.Event] = None
        self._grace: Optional[float] = None
        self._stopping = False
        self.stop_completed = False  # server.stop() ran to the end on the loop
        self._thread = threading.Thread(target=self._run, args=(servicer, port, host), daemon=True,
                                        name="grpc-aio-server")
        self._thread.start()
        self._ready.wait(60)
        if self._err is not None:
            raise self._err
        if self.bound_port is None:
            raise RuntimeError("gRPC aio server did not start")

    def _run(self, servicer, port, host):
        asyncio.set_event_loop(self.loop)

        async def main():
            self._server = grpc.aio.server(options=[("grpc.max_receive_message_length", 64 << 20)])
            add_servicer(self._server, servicer)
            self.bound_port = self._server.add_insecure_port(f"{host}:{port}")
            await self._server.start()
            self._stop_ev = asyncio.Event()
            self._ready.set()
            term = asyncio.ensure_future(self._server.wait_for_termination())
            req = asyncio.ensure_future(self._stop_ev.wait())
            done, _ = await asyncio.wait({term, req}, return_when=asyncio.FIRST_COMPLETED)
            if req in done:
                await self._server.stop(self._grace)
                self.stop_completed = True
            else:
                log.warning("gRPC aio server terminated without stop()")
            for t in (term, req):
                t.cancel()

        try:
            self.loop.run_until_complete(main())
        except BaseException as e:  # noqa: BLE001 - reported to the constructor / stop()
            self._err = e
            self._ready.set()
            log.error("gRPC aio server loop ended with %r", e)
        finally:
            try:
                if self._server is not None and not self.stop_completed:  # main did not get to stop it (the loop
                    # was stopped from outside, or main failed): stop it here, while the loop still runs tasks,
                    # so grpc's own finaliser never schedules onto a closed loop
                    self.loop.run_until_complete(asyncio.wait_for(self._server.stop(0), 10))
                # servicer coroutines of calls the stop cancelled: finish them here, not in a dead loop
                pending = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
                for t in pending:
                    t.cancel()
                if pending:
                    self.loop.run_until_complete(asyncio.wait_for(asyncio.gather(*pending, return_exceptions=True),
                                                                  10))
            except BaseException as e:  # noqa: BLE001 - best effort; the thread must end
                log.warning("gRPC aio server loop clean-up: %r", e)
            if not self.loop.is_running():
                self.loop.close()
            self._stopped = True

    def stop(self, grace: Optional[float] = None):
        """Ask the loop to stop the server (it runs ``server.stop(grace)`` itself); ``.wait(timeout)`` joins the
        loop thread. A loop that already ended has nothing to stop."""
        th = self._thread
        self._stopping = True
        self._grace = grace
        if th.is_alive() and self._stop_ev is not None and not self.loop.is_closed():
            try:
                self.loop.call_soon_threadsafe(self._stop_ev.set)
            except RuntimeError:  # closed between the check and the call
                pass

        class _Done:
            def wait(self, timeout: Optional[float] = None) -> bool:
                th.join(timeout)
                return not th.is_alive()
        return _Done()

    def wait_for_termination(self, timeout: Optional[float] = None) -> bool:
        self._thread.join(timeout)
        return not self._thread.is_alive()


class Stub:
    """Client stub (what grpc_tools would generate)."""

    def __init__(self, channel: grpc.Channel):
        self.Generate = channel.unary_unary(f"/{SERVICE}/Generate", request_serializer=GenerateRequest.SerializeToString,
                                            response_deserializer=GenerateResponse.FromString)
        self.GenerateStream = channel.unary_stream(f"/{SERVICE}/GenerateStream",
                                                   request_serializer=GenerateRequest.SerializeToString,
                                                   response_deserializer=Token.FromString)
        self.Stats = channel.unary_unary(f"/{SERVICE}/Stats", request_serializer=StatsRequest.SerializeToString,
                                         response_deserializer=StatsResponse.FromString)


# ------------------------------------------------------------------------------ servicers
def _resolve(fut, value):
    if not fut.done():
        fut.set_result(value)


def _fanout(items):
    for q, t in items:
        q.put_nowait(t)


class _LoopSink:
    """Driver-thread -> event-loop hand-off of one step's stream tokens in ONE call_soon_threadsafe
    (``Handle.sink``): 64 streams cost one loop wake-up per step, not 64."""

    def __init__(self, loop):
        self.loop = loop

    def __call__(self, items):
        try:
            self.loop.call_soon_threadsafe(_fanout, items)
        except RuntimeError:  # the server stopped and closed its loop: the streams' receivers are gone
            pass


class EngineServicer:
    """Direct servicer on the TP leader (coroutine handlers: :func:`serve` runs it on a ``grpc.aio`` server)."""

    def __init__(self, driver, tokenizer):
        self.driver = driver
        self.tok = tokenizer
        self._sinks = {}  # event loop -> _LoopSink

    def _prompt_ids(self, req):
        from ..utils.tokenizer import encode

        if len(req.prompt_token_ids):
            return list(req.prompt_token_ids)
        return encode(self.tok, req.prompt)

    async def Generate(self, req, ctx):
        try:
            params = _params(req)
        except ValueError as e:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        remaining = ctx.time_remaining()  # gRPC deadline -> server-side deadline on every rank
        h = self.driver.submit(self._prompt_ids(req), params, deadline_s=remaining,
                               on_done=lambda h_: loop.call_soon_threadsafe(_resolve, fut, h_))
        try:
            await (asyncio.wait_for(fut, remaining) if remaining is not None else fut)
        except asyncio.TimeoutError:
            self.driver.abort(h.rid)
            await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
        except asyncio.CancelledError:  # the client went away
            self.driver.abort(h.rid)
            raise
        if h.finish_reason == "error":
            await ctx.abort(grpc.StatusCode.UNAVAILABLE, h.error or "engine failure")
        if h.finish_reason == "deadline":  # the driver's copy of the call's deadline fired first: same status as above
            await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
        m = h.metrics or {}
        return GenerateResponse(prompt=req.prompt, continuation=self.tok.decode(h.output_ids), request_id=req.request_id,
                                token_ids=h.output_ids, finish_reason=h.finish_reason,
                                ttft_s=float(m.get("ttft_s", 0.0) or 0.0), e2e_s=float(m.get("e2e_s", 0.0) or 0.0))

    async def GenerateStream(self, req, ctx):
        try:
            params = _params(req)
        except ValueError as e:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        sink = self._sinks.get(loop)
        if sink is None:
            sink = self._sinks[loop] = _LoopSink(loop)
        # tokens and the final None reach the queue in the driver's order (one batch per step, batches FIFO)
        h = self.driver.submit(self._prompt_ids(req), params, deadline_s=ctx.time_remaining(), sink=sink, sink_q=q)
        from ..utils.tokenizer import StreamDecoder

        dec = StreamDecoder(self.tok)  # one short-window decode per token, not the whole prefix again
        try:
            while True:
                t = await q.get()
                if t is None:
                    break
                yield Token(token_id=t, text=dec.push(t), finished=False)
        except asyncio.CancelledError:
            if not h.done.is_set():
                self.driver.abort(h.rid)
            raise
        if h.finish_reason == "error":
            await ctx.abort(grpc.StatusCode.UNAVAILABLE, h.error or "engine failure")
        if h.finish_reason == "deadline":  # the tokens so far were streamed; the call ends as its deadline says
            await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
        yield Token(token_id=-1, text=dec.flush(), finished=True, finish_reason=h.finish_reason)

    async def Stats(self, req, ctx):
        st = dict(self.driver.engine.stats)
        st["healthy"] = self.driver.error is None
        if self.driver.error is not None:
            st["error"] = str(self.driver.error)
        return StatsResponse(json=json.dumps(st))


class BrokerServicer:
    """gRPC front-end of the pub/sub path: enqueue on the broker, wait for the correlated reply."""

    def __init__(self, broker, default_timeout: float = 600.0):
        self.broker = broker
        self.timeout = default_timeout
        self.stats = {"requests": 0, "timeouts": 0}

    @staticmethod
    def _body(req, rid, stream=False, deadline_s=None):
        from .protocol import Request

        # deadline_s: the call's remaining time, so the consumer stops generating when nobody waits any more
        return Request(prompt=req.prompt, max_new_tokens=req.max_new_tokens or 20, is_greedy=req.is_greedy,
                       temperature=req.temperature or 1.0, top_p=req.top_p or 0.95, top_k=req.top_k or 50,
                       request_id=rid, seed=req.seed or None, ignore_eos=req.ignore_eos, stream=stream,
                       prompt_token_ids=list(req.prompt_token_ids) or None, deadline_s=deadline_s)

    def Generate(self, req, ctx):
        from .broker import PQUEUE, reply_key
        from .protocol import new_request_id

        rid = req.request_id or new_request_id()
        remaining = ctx.time_remaining()
        body = self._body(req, rid, deadline_s=remaining)
        t0 = time.perf_counter()
        self.broker.lpush(PQUEUE, body.model_dump_json(exclude_none=True))
        self.stats["requests"] += 1
        msg = self.broker.brpop(reply_key(rid), timeout=remaining if remaining else self.timeout)
        if msg is None:
            self.stats["timeouts"] += 1
            ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "no reply from consumer")
        d = json.loads(msg)
        if d.get("finish_reason") == "deadline":  # the consumer stopped at the deadline this call sent along
            ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
        return GenerateResponse(prompt=d.get("prompt", ""), continuation=d.get("continuation", ""), request_id=rid,
                                token_ids=d.get("token_ids") or [], finish_reason=d.get("finish_reason", ""), ttft_s=float(d.get("ttft_s") or 0.0),
                                e2e_s=float(time.perf_counter() - t0))

    def GenerateStream(self, req, ctx):
        """Streams through the broker: the consumer pushes the tokens of every engine step to the
        request's reply list as they are sampled ({"token_ids": [...], "text": ...}), then a final
        message with "finished"; each token becomes one Token message here."""
        from .broker import PQUEUE, reply_key
        from .protocol import new_request_id

        rid = req.request_id or new_request_id()
        remaining = ctx.time_remaining()
        self.broker.lpush(PQUEUE, self._body(req, rid, stream=True, deadline_s=remaining).model_dump_json(
            exclude_none=True))
        self.stats["requests"] += 1
        deadline = time.monotonic() + (remaining if remaining else self.timeout)
        while True:
            msg = self.broker.brpop(reply_key(rid), timeout=max(0.001, deadline - time.monotonic()))
            if msg is None:
                self.stats["timeouts"] += 1
                ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "no reply from consumer")
            d = json.loads(msg)
            if d.get("error"):
                ctx.abort(grpc.StatusCode.UNAVAILABLE, d["error"])
            if d.get("finished") and d.get("finish_reason") == "deadline":
                ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
            if d.get("finished"):
                yield Token(token_id=-1, text=d.get("text", ""), finished=True, finish_reason=d.get("finish_reason", ""))
                return
            ids = d.get("token_ids") or []
            for j, t in enumerate(ids):
                yield Token(token_id=int(t), text=d.get("text", "") if j == len(ids) - 1 else "", finished=False)

    def Stats(self, req, ctx):
        return StatsResponse(json=json.dumps(self.stats))


class AioBrokerServicer(BrokerServicer):
    """The pub/sub front-end on a ``grpc.aio`` server with an asyncio RESP client (:class:`AsyncRedisClient`):
    every in-flight request is a coroutine on one event loop instead of a pool thread blocked in its own BRPOP.
    The thread-pool form spent ~100 ms of interpreter-lock hand-offs turning a cohort of 64 replies into 64 new
    requests (bench/pubsub_rtt.py: 131 ms vs 30 ms with clients on the broker directly), and the engine idled for
    the cohort meanwhile (profiles/r6_pubsub). Same wire behaviour as :class:`BrokerServicer`."""

    def __init__(self, host: str, port: int, default_timeout: float = 600.0):
        from .broker import AsyncRedisClient

        super().__init__(None, default_timeout)
        self.client = AsyncRedisClient(host, port)

    async def Generate(self, req, ctx):
        from .broker import PQUEUE, reply_key
        from .protocol import new_request_id

        rid = req.request_id or new_request_id()
        t0 = time.perf_counter()
        remaining = ctx.time_remaining()
        await self.client.lpush(PQUEUE, self._body(req, rid, deadline_s=remaining).model_dump_json(exclude_none=True))
        self.stats["requests"] += 1
        msg = await self.client.brpop(reply_key(rid), timeout=remaining if remaining else self.timeout)
        if msg is None:
            self.stats["timeouts"] += 1
            await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "no reply from consumer")
        d = json.loads(msg)
        if d.get("finish_reason") == "deadline":  # the consumer stopped at the deadline this call sent along
            await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
        return GenerateResponse(prompt=d.get("prompt", ""), continuation=d.get("continuation", ""), request_id=rid,
                                token_ids=d.get("token_ids") or [], finish_reason=d.get("finish_reason", ""),
                                ttft_s=float(d.get("ttft_s") or 0.0), e2e_s=float(time.perf_counter() - t0))

    async def GenerateStream(self, req, ctx):
        from .broker import PQUEUE, reply_key
        from .protocol import new_request_id

        rid = req.request_id or new_request_id()
        remaining = ctx.time_remaining()
        await self.client.lpush(PQUEUE, self._body(req, rid, stream=True, deadline_s=remaining).model_dump_json(
            exclude_none=True))
        self.stats["requests"] += 1
        deadline = time.monotonic() + (remaining if remaining else self.timeout)
        while True:
            msg = await self.client.brpop(reply_key(rid), timeout=max(0.001, deadline - time.monotonic()))
            if msg is None:
                self.stats["timeouts"] += 1
                await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "no reply from consumer")
            d = json.loads(msg)
            if d.get("error"):
                await ctx.abort(grpc.StatusCode.UNAVAILABLE, d["error"])
            if d.get("finished") and d.get("finish_reason") == "deadline":
                await ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "generation deadline exceeded")
            if d.get("finished"):
                yield Token(token_id=-1, text=d.get("text", ""), finished=True, finish_reason=d.get("finish_reason", ""))
                return
            ids = d.get("token_ids") or []
            for j, t in enumerate(ids):
                yield Token(token_id=int(t), text=d.get("text", "") if j == len(ids) - 1 else "", finished=False)

    async def Stats(self, req, ctx):
        return StatsResponse(json=json.dumps(self.stats))
