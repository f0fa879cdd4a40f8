"""Prefill GEMM A/B in one process on random data: hipBLASLt (torch.matmul), the in-tree gemm_big, and the
ping-pong prototype variants of bench/proto/pp_gemm.hip (built to bench/proto/libpp.so).

usage: python bench/pp_probe.py [--m 8192] [--shapes qkv,o,gate_up,down,cube] [--vars 0,1,2,3,4,5] [--rounds 5]
Prints one JSON line per (shape, arm) with the median / best TFLOP/s over interleaved rounds and the max
error against torch.matmul.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
          "cube": (8192, 8192), "gpt2_qkv": (4800, 1600), "gpt2_down": (1600, 6400),
          "tp8_qkv": (1536, 4096), "tp8_o": (4096, 512), "tp8_up": (2752, 4096), "tp8_down": (4096, 1376)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="8192")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--vars", default="0,1,2,3,4,5")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=os.path.join(ROOT, "bench", "proto", "libpp.so"))
    ap.add_argument("--gm", type=int, default=4)
    ap.add_argument("--no-big", action="store_true")
    ap.add_argument("--no-lib", action="store_true")
    a = ap.parse_args()
    pp = ctypes.CDLL(a.lib)
    pp.pp_gemm.restype = ctypes.c_int
    pp.pp_gemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    H = None
    if not a.no_big:
        from llmss_amd.ops import hip as H  # noqa: N812
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    variants = [int(v) for v in a.vars.split(",") if v != ""]
    for M in [int(m) for m in a.m.split(",")]:
        for name in a.shapes.split(","):
            N, K = SHAPES[name] if name != "cube" else (M, M)
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / 16).to(torch.bfloat16)
            ref = torch.matmul(x, w.t())
            scale = ref.float().abs().max().item()
            ys = {}
            arms = {}

            def lib_fn(y):
                torch.matmul(x, w.t(), out=y)
            if not a.no_lib:
                arms["lib"] = lib_fn
            if H is not None:
                def big_fn(y):
                    H.linear(x, w, out=y)
                arms["big"] = big_fn
            for v in variants:
                def pp_fn(y, v=v):
                    rc = pp.pp_gemm(v, x.data_ptr(), K, w.data_ptr(), K, None, y.data_ptr(), N, M, N, K, 0, 0, a.gm,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    if rc:
                        raise RuntimeError(f"pp_gemm rc={rc}")
                arms[f"pp{v}"] = pp_fn
            err = {}
            for k, fn in arms.items():
                y = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
                fn(y)
                torch.cuda.synchronize()
                err[k] = (y.float() - ref.float()).abs().max().item() / scale
                ys[k] = y
            times = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    y = ys[k]
                    fn(y)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.iters):
                        fn(y)
                    e.record()
                    torch.cuda.synchronize()
                    times[k].append(s.elapsed_time(e) / a.iters * 1e3)
            fl = 2.0 * M * N * K
            for k in arms:
                med, best = statistics.median(times[k]), min(times[k])
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "arm": k, "us_med": round(med, 1),
                                  "tf_med": round(fl / med / 1e6, 1), "tf_best": round(fl / best / 1e6, 1),
                                  "rel_err": round(err[k], 5)}), flush=True)
            del x, w, ref, ys


if __name__ == "__main__":
    main()
