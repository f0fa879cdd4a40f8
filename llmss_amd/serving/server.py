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
    add_engine_args(p)
    args = p.parse_args(argv)
    driver, tok, _ = build_driver(args.model, args)
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


if __name__ == "__main__":
    main()
