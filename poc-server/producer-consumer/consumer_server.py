"""Pub/sub consumer (API-compatible with the reference consumer_server.py), launched with
``torchrun --nproc_per_node N consumer_server.py --pretrained_model_path ...``: rank 0 pops
requests from Redis ``pqueue`` and all ranks decode them together with continuous batching over
RCCL tensor parallelism; replies go to ``squeue`` (``squeue:<request_id>`` when the request has
an id). ``--model_type`` (documented in the reference README but rejected by its argparse, Q15)
is accepted and checked against the checkpoint. ``--grpc_port`` additionally serves gRPC
directly from rank 0."""
import os
import sys
import threading
from argparse import ArgumentParser

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))


def get_args(argv=None):
    parser = ArgumentParser()
    consumer_group = parser.add_argument_group("consumer")
    consumer_group.add_argument("--pretrained_model_path", type=str, required=True)
    consumer_group.add_argument("--model_type", type=str, default=None)
    consumer_group.add_argument("--grpc_port", type=int, default=0)
    # durable hand-off: in-flight requests sit in pqueue:processing:<id> until answered; a consumer restarted
    # with the same id re-queues what its previous incarnation left there
    consumer_group.add_argument("--consumer_id", type=str, default="0")
    consumer_group.add_argument("--reply_ttl_s", type=float, default=300.0,
                                help="TTL of every reply list (Redis EXPIRE): replies nobody pops are deleted")
    broker_group = parser.add_argument_group("broker")
    broker_group.add_argument("--redis_host", type=str, default="127.0.0.1")
    broker_group.add_argument("--redis_port", type=int, default=20000)
    from llmss_amd.serving.launch import add_engine_args

    add_engine_args(parser)
    return parser.parse_args(argv)


def main(argv=None):
    from llmss_amd.serving.broker import RedisBroker
    from llmss_amd.serving.consumer import Consumer
    from llmss_amd.serving.grpc_api import EngineServicer, serve
    from llmss_amd.serving.launch import build_driver

    args = get_args(argv)
    driver, tok, model = build_driver(args.pretrained_model_path, args)
    if args.model_type and args.model_type not in (model.cfg.model_type, "gpt_bigcode" if model.cfg.model_type == "gpt_bigcode" else None):
        raise SystemExit(f"--model_type {args.model_type} does not match checkpoint type {model.cfg.model_type}")
    # --dp N with torchrun: world = N replicas x TP; every replica leader pulls from the same broker
    if driver.leader:
        print(f"{model.cfg.model_type} setup is done.", flush=True)
        Consumer(driver, tok, RedisBroker(args.redis_host, args.redis_port), consumer_id=args.consumer_id,
                 reply_ttl_s=args.reply_ttl_s).start()
        if args.grpc_port:
            serve(EngineServicer(driver, tok), args.grpc_port)
    driver.run()  # blocks forever on every rank (leader: driver loop in this thread)


if __name__ == "__main__":
    main()
