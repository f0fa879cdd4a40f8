"""Repeat-run determinism probe for the tiled / mid GEMM kernels: the same call on NaN-filled outputs
N times must give bit-identical results that match the fp32 reference (catches cross-tile write
races and unwritten elements that a recycled output buffer would hide)."""
import sys

import torch

sys.path.insert(0, ".")
from llmss_amd.ops import hip as H  # noqa: E402
from llmss_amd.ops import reference as R  # noqa: E402


def main():
    dev = torch.device("cuda")
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    bad = 0
    for (M, N, K) in [(200, 4800, 1600), (700, 1312, 192), (512, 1536, 4096), (333, 2048, 1024)]:
        torch.manual_seed(0)
        x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
        ref = R.linear(x.float(), w.float(), b.float(), act="gelu_tanh")
        for tile in (1, 2, 3, 5, 6, 8, 9, 10, 11, 12):
            for stages in (2, 3, 4):
                for split in (1, 3):
                    hint = (tile | ({2: 0, 3: 16, 4: 32, 6: 48}[stages])) << 8
                    first = None
                    for r in range(reps):
                        y = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev)
                        H.linear(x, w, b, act="gelu_tanh", nt_hint=hint, split_hint=split, out=y)
                        if first is None:
                            first = y.clone()
                            err = (y.float() - ref).abs() - (2e-2 + 0.02 * ref.abs())
                            nb = int((~(err <= 0)).sum())
                            if nb:
                                rows = (~(err <= 0)).nonzero()[:, 0].unique().tolist()
                                print(f"WRONG M{M} N{N} K{K} tile{tile} ns{stages} split{split}: {nb} bad, rows {rows[:12]}",
                                      flush=True)
                                bad += 1
                        elif not torch.equal(y.view(torch.int16), first.view(torch.int16)):
                            d = (y.view(torch.int16) != first.view(torch.int16)).nonzero()
                            print(f"NONDET M{M} N{N} K{K} tile{tile} ns{stages} split{split} rep{r}: {len(d)} differ, "
                                  f"rows {d[:, 0].unique().tolist()[:12]}", flush=True)
                            bad += 1
                            break
        print(f"M{M} N{N} K{K} done", flush=True)
    print("BAD", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
