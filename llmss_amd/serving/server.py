"""Direct gRPC server on the tensor-parallel leader (no broker).

    torchrun --nproc_per_node N -m llmss_amd.serving.server --model /path/or/preset --grpc_port 50051
"""
from __future__ import annotations

import argparse
import signal
import threading

from .grpc_api import EngineServicer, serve
from .launch import add_engine_args, build_driver


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", "--pretrained_model_path", dest="model", required=True)
    p.add_argument("--grpc_host", default="0.0.0.0")
    p.add_argument("--grpc_port", type=int, default=50051)
    p.add_argument("--broker_port", type=int, default=20001,
                   help="with torchrun --dp > 1: port of the in-process broker on rank 0 that the replicas pull from")
    add_engine_args(p)
    args = p.parse_args(argv)
    driver, tok, _ = build_driver(args.model, args)
    if getattr(driver.tp, "dp", 1) > 1:  # multi-process data parallelism: replicas pull from one broker
        return _serve_replicas(driver, tok, args)
    if driver.leader:
        driver.start()
        server = serve(EngineServicer(driver, tok), args.grpc_port, args.grpc_host)
        print(f"llmss gRPC Generate serving on {args.grpc_host}:{server.bound_port} (tp={driver.tp.size})", flush=True)
        stop = threading.Event()
        signal.signal(signal.SIGTERM, lambda *a: stop.set())
        try:
            stop.wait()
        except KeyboardInterrupt:
            pass
        server.stop(5)
        driver.stop()
    else:
        driver.run()


def _serve_replicas(driver, tok, args):
    """torchrun world = dp x tp: global rank 0 hosts a broker and the gRPC front-end (AioBrokerServicer);
    every replica leader runs a Consumer on that broker (BRPOP = load balancing, replies correlated
    by request id); followers run their replica's driver loop."""
    import torch.distributed as dist

    from .broker import MiniRedisServer, RedisBroker
    from .consumer import Consumer
    from .grpc_api import AioBrokerServicer

    g = driver.tp
    broker_srv = None
    if g.global_rank == 0:
        broker_srv = MiniRedisServer("127.0.0.1", args.broker_port).start()
    dist.barrier()  # the broker is listening before replicas connect
    if driver.leader:
        # one processing list per replica (durable hand-off, consumer.py)
        Consumer(driver, tok, RedisBroker("127.0.0.1", args.broker_port), consumer_id=f"replica{g.replica}").start()
    if g.global_rank == 0:
        server = serve(AioBrokerServicer("127.0.0.1", args.broker_port), args.grpc_port, args.grpc_host)
        print(f"llmss gRPC Generate on {args.grpc_host}:{server.bound_port}: {g.dp} replicas x tp={g.size}", flush=True)
    driver.run()


if __name__ == "__main__":
    main()
