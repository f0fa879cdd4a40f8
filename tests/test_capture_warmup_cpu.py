"""Every collective a captured decode graph issues was issued eagerly before the capture: a
native RCCL communicator sets up each algorithm's peer connections lazily on first use, which must never happen
inside a HIP graph capture. The engine warms every (bucket, sampler mode) eagerly before capture_graphs captures it,
and every A/B schedule (tbo / rsag / col) once per bucket with the first sampler mode before its captures. This CPU
test runs those same forwards with a recording TP group (a fake TP=2 group that models collectives: the
schedules that need a communicator take their real code paths) and checks, per bucket, sampler mode and schedule,
that the captured forward's collective signatures (kind, element count, dtype) are a subset of what the warm-ups
issued. CPU only."""
import torch

from llmss_amd.engine import LLMEngine
from llmss_amd.engine.engine import _DecodeBuffers
from llmss_amd.models.config import get_preset
from llmss_amd.models.decoder import DecoderLM
from llmss_amd.models.weights import random_weights
from llmss_amd.parallel.dist import TPGroup


class RecordingTP(TPGroup):
    def __init__(self):
        super().__init__(0, 2, fake=True, sim_comm=(1.0, 1.0))
        self.replicate_gather = True
        self.log = []

    def _rec(self, kind, t):
        self.log.append((kind, int(t.numel()), str(t.dtype)))

    def all_reduce(self, t):
        self._rec("all_reduce", t)
        return super().all_reduce(t)

    def all_gather_last_dim(self, t):
        self._rec("all_gather", t)
        return super().all_gather_last_dim(t)

    def all_gather_rows(self, t):
        self._rec("all_gather", t)
        return super().all_gather_rows(t)

    def reduce_scatter_rows(self, t):
        self._rec("reduce_scatter", t)
        return super().reduce_scatter_rows(t)


def test_warmup_covers_every_captured_collective(monkeypatch):
    monkeypatch.setenv("LLMSS_TP_COL", "2")  # make the column schedule applicable (forced mode) for the check
    cfg = get_preset("tiny-llama", hidden_size=256, num_heads=4, num_kv_heads=2, head_dim=64, rotary_dim=64,
                     intermediate_size=512, max_position_embeddings=256, num_layers=2)
    tp = RecordingTP()
    m = DecoderLM(cfg, random_weights(cfg, 2, 0, dtype=torch.float32, seed=5, std=0.05), tp)
    m.col_mode = "auto"  # the A/B decides per bucket (forced mode would run it in every forward)
    e = LLMEngine(m, max_num_seqs=24, block_size=16, use_graphs=False, autotune=False, graph_buckets=[1, 8, 16, 24])
    buf = e.buf = _DecodeBuffers(e.buckets[-1], e.max_blocks, torch.device("cpu"))
    buf.d_i64.zero_()
    buf.slots.fill_(-1)
    buf.d_i32.zero_()
    buf.topk.fill_(1)
    buf.d_f32.zero_()
    modes = e._decode_modes()
    assert modes == (True, False)  # vocab-parallel: both samplers are captured

    def issued(b, d, name=None):
        tp.log.clear()
        if name is None:
            e._decode_forward(b, buf, dist=d)
        else:
            with e._schedule(b, name):
                e._decode_forward(b, buf, dist=d)
        return set(tp.log)

    applicable = {"tbo": lambda b: b >= 2,
                  "rsag": m.rsag_ok, "col": lambda b: m.col_ok(m.w.layers[0].o) and m.col_ok(m.w.layers[0].down)}
    checked, needed_alt_warm = 0, set()
    for b in e.buckets:
        warm_one = {d: issued(b, d) for d in modes}  # capture_graphs' eager passes
        for d in modes:  # capture_graphs: the one-all-reduce graph
            assert issued(b, d) <= warm_one[d]
        for name, ok in applicable.items():
            if not ok(b):
                continue
            warm_alt = issued(b, modes[0], name)  # the A/B's warm stage: first sampler mode only
            for d in modes:
                cap = issued(b, d, name)
                missing = cap - warm_one[d] - warm_alt
                assert not missing, (b, d, name, missing)
                checked += 1
                if cap - warm_one[d]:
                    needed_alt_warm.add(name)
    assert checked >= 12
    # the schedules issue collectives of their own sizes (half batches, row shards, column chunks): without the A/B's
    # eager warm-up those would first run inside a capture
    assert needed_alt_warm == {"tbo", "rsag", "col"}, needed_alt_warm
