"""Cost of real RCCL collectives inside the decode HIP graphs, on one GPU.

usage: python bench/rccl_graph_probe.py [--tp 8] [--steps 2]

The rank-0 shard of Llama-2-7B at TP=N (batch 64 * N) runs the bench step twice: on a fake group (no
collectives: the per-rank compute time) and on a ONE-member RCCL communicator that claims N ranks (every
all-reduce / all-gather of the step is issued through torch.distributed / RCCL exactly as at TP=N and captured
into the decode graphs, but with one member the sum is the identity). The difference is what the collective
launches, their stream hand-offs inside the graphs and RCCL's own kernels cost before any xGMI transfer.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from llmss_amd.parallel.dist import TPGroup  # noqa: E402


class OneMemberTP(TPGroup):
    """TP=N shard plan over a 1-rank communicator: all-gathers return N copies of the local shard."""

    def all_gather_last_dim(self, t):
        out = torch.empty_like(t.contiguous())
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return torch.cat([out] * self.size, -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--model", default="llama2-7b")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    args = argparse.Namespace(gpus=1, steps=a.steps, warmup=1, batch_per_gpu=64, prompt_len=128, gen_len=128,
                              fp8=False, kv_dtype="bf16", greedy=False, no_graphs=False, simulate_tp=a.tp,
                              sim_comm="")

    def progress(msg):
        print(f"[probe] {msg}", file=sys.stderr, flush=True)

    fake = TPGroup(0, a.tp, fake=True)
    fake.replicate_gather = True  # same gathered widths as the RCCL group below
    for name, tp in (("fake group (no collectives)", fake),
                     ("one-member RCCL group", OneMemberTP(0, a.tp, group=dist.group.WORLD))):
        r = bench.run_config(args, a.model, tp, 64 * a.tp, progress)
        print(json.dumps({"group": name, "tokens_per_s": r["value"], "ms_per_step": r["ms_per_step"],
                          "p50_tpot_ms": r["p50_tpot_ms"], "p50_ttft_ms": r["p50_ttft_ms"]}), flush=True)
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
