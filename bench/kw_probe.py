"""Decode GEMM A/B (M <= 64) in one process: the in-tree plans (best of the autotuner's candidate list) against
the K-split-wave prototype of bench/proto/kw_gemm.hip (bench/proto/libkw.so), weights rotated through > 600 MB so
every call streams them from HBM as a decode step does. Split-K arms (S > 1) leave fp32 slabs for the consumer
and are charged the consumer's slab reads (ops/autotune.py _SLAB_READ_BPS), like the autotuner charges ours.

usage: python bench/kw_probe.py [--m 64] [--shapes qkv,o,gate_up,down] [--vars 0,1,2] [--splits 1,2,4]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
          "gpt2_qkv": (4800, 1600), "gpt2_o": (1600, 1600), "gpt2_up": (6400, 1600), "gpt2_down": (1600, 6400),
          "tp8_qkv": (1536, 4096), "tp8_o": (4096, 512), "tp8_up": (2752, 4096), "tp8_down": (4096, 1376)}


def main():
    from gemm_bench import timeit

    from llmss_amd.ops import autotune as A
    from llmss_amd.ops import hip as H

    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="64")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--vars", default="0,1,2,3,4,5,6,7,8,9,10,11")
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--no-base", action="store_true")
    ap.add_argument("--lib", default=os.path.join(ROOT, "bench", "proto", "libkw.so"))
    a = ap.parse_args()
    kw = ctypes.CDLL(a.lib)
    kw.kw_gemm.restype = ctypes.c_int
    kw.kw_gemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    H.reserve_workspace(dev, 64 << 20)
    part = torch.empty(16 << 20, dtype=torch.float32, device=dev)
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        wbytes = N * K * 2
        ncopy = max(2, int(600e6 // wbytes) + 1)
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
        for M in [int(m) for m in a.m.split(",")]:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ref = (x.float() @ ws[0].float().t())
            res = {"shape": name, "M": M, "N": N, "K": K}
            if not a.no_base:
                best = None
                for nt, sp in [(0, 0)] + A.candidates(M, N, K, False, False):
                    try:
                        t = timeit(lambda i: H.linear(x, ws[i % ncopy], None, out=y, nt_hint=nt, split_hint=sp),
                                   iters=30)
                    except (ValueError, RuntimeError):
                        continue
                    if best is None or t < best[0]:
                        best = (t, nt, sp)
                res["base_us"], res["base_plan"] = round(best[0], 2), best[1:]
                res["base_TBps"] = round(wbytes / best[0] / 1e6, 2)
            for v in [int(s) for s in a.vars.split(",") if s]:
                for S in [int(s) for s in a.splits.split(",")]:
                    def run(i, v=v, S=S):
                        rc = kw.kw_gemm(v, x.data_ptr(), K, ws[i % ncopy].data_ptr(), K, y.data_ptr(), N,
                                        part.data_ptr(), M, N, K, S,
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                        if rc:
                            raise RuntimeError(f"kw rc={rc}")
                    run(0)
                    torch.cuda.synchronize()
                    got = y.float() if S == 1 else part[:S * M * N].view(S, M, N).sum(0)
                    err = ((got - ref).abs().max() / ref.abs().max()).item()
                    t = timeit(run, iters=30)
                    charge = (S * M * N * 4 / A._SLAB_READ_BPS * 1e6) if S > 1 else 0.0
                    res[f"kw{v}_s{S}"] = [round(t, 2), round(t + charge, 2), round(err, 4)]
            cands = {k: v[1] for k, v in res.items() if k.startswith("kw") and v[2] < 0.02}
            if cands:
                k = min(cands, key=cands.get)
                res["kw_best"] = [k, cands[k], round(wbytes / cands[k] / 1e6, 2)]
            print(json.dumps(res), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
