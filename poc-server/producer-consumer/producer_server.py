"""Pub/sub producer (API-compatible with the reference producer_server.py): HTTP POST /generate
-> Redis list ``pqueue`` -> consumer -> reply. Same flags; additions: ``--grpc_port`` (gRPC
Generate front-end on the same broker) and ``--embedded_redis`` (start a built-in RESP server
when no redis-server is available)."""
import os
import sys
from argparse import ArgumentParser

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))


def get_args(argv=None):
    parser = ArgumentParser()
    producer_group = parser.add_argument_group("producer")
    producer_group.add_argument("--fastapi_host", type=str, default="127.0.0.1")
    producer_group.add_argument("--fastapi_port", type=int, default=8000)
    producer_group.add_argument("--grpc_port", type=int, default=0, help="also serve gRPC Generate (0 = off)")
    broker_group = parser.add_argument_group("broker")
    broker_group.add_argument("--redis_host", type=str, default="127.0.0.1")
    broker_group.add_argument("--redis_port", type=int, default=20000)
    broker_group.add_argument("--embedded_redis", action="store_true", help="run a built-in RESP server on redis_port")
    return parser.parse_args(argv)


def main(argv=None):
    import uvicorn

    from llmss_amd.serving.broker import MiniRedisServer, RedisBroker
    from llmss_amd.serving.grpc_api import AioBrokerServicer, serve
    from llmss_amd.serving.producer import create_app

    args = get_args(argv)
    if args.embedded_redis:
        MiniRedisServer(args.redis_host, args.redis_port).start()
    broker = RedisBroker(args.redis_host, args.redis_port)
    if args.grpc_port:
        serve(AioBrokerServicer(args.redis_host, args.redis_port), args.grpc_port)
    uvicorn.run(create_app(broker), host=args.fastapi_host, port=args.fastapi_port)


if __name__ == "__main__":
    main()
