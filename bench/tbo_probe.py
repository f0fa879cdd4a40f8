"""Decode-step graph replay time of the micro-batch overlap schedule vs the single-batch step
(simulated TP=8 Llama-2-7B shard, fewer layers), per diagnostic variant of LLMSS_TBO_DIAG."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llmss_amd.engine import LLMEngine
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights
    from llmss_amd.parallel.dist import TPGroup

    dev = torch.device("cuda", 0)
    cfg = get_preset("llama2-7b", num_layers=int(os.environ.get("LAYERS", "8")), max_position_embeddings=512)
    tp = TPGroup(0, 8, fake=True, sim_comm=tuple(float(v) for v in os.environ.get("SIM", "0.1,100000").split(",")))
    w = random_weights(cfg, 8, 0, device=dev, dtype=torch.bfloat16, seed=0)
    for variant in os.environ.get("VARIANTS", "off,on,norecord,onestream").split(","):
        os.environ["LLMSS_TBO_DIAG"] = variant
        m = DecoderLM(cfg, w, tp)
        m.tbo_min = 0 if variant == "off" else 64
        B = 512
        eng = LLMEngine(m, max_num_seqs=B, max_model_len=512, block_size=16, use_graphs=True, autotune=False,
                        graph_buckets=[B])
        buf = eng.buf
        buf.ctx[:B] = 200
        buf.bt[:B] = torch.arange(B * eng.max_blocks, device=dev, dtype=torch.int32).view(B, -1)[:, :] % eng.num_blocks
        buf.slots[:B] = -1
        g = eng.graphs[B]
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 5 * 1e3)
        print(json.dumps({"variant": variant, "layers": cfg.num_layers, "batch": B, "sim": os.environ.get("SIM"),
                          "graph_step_us": round(best, 1)}), flush=True)
        del eng, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
