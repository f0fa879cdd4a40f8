"""CPU parity of the family-agnostic decoder vs HF transformers at fp32 (tiny random checkpoints
loaded through the native safetensors reader), incl. paged-KV greedy decoding through the engine."""
import os

import pytest
import torch

from helpers import FAMILIES, save_hf_model
from llmss_amd.engine import LLMEngine, SamplingParams
from llmss_amd.models.config import ModelConfig, get_preset, preset_names
from llmss_amd.models.decoder import DecoderLM, StepInput
from llmss_amd.models.weights import load_hf_weights, random_weights, shard_plan
from llmss_amd.utils.checkpoint import CheckpointReader, weight_files


@pytest.fixture(scope="module")
def ckpts(tmp_path_factory):
    out = {}
    for name in FAMILIES:
        d = str(tmp_path_factory.mktemp(name))
        out[name] = (d, save_hf_model(name, d))
    return out


def _load(d, tp=1, rank=0):
    cfg = ModelConfig.from_pretrained(d)
    w = load_hf_weights(cfg, CheckpointReader(weight_files(d)), tp, rank, device="cpu", dtype=torch.float32)
    return cfg, w


@pytest.mark.parametrize("name", FAMILIES)
def test_prefill_logits_match_hf(ckpts, name):
    d, hf = ckpts[name]
    cfg, w = _load(d)
    m = DecoderLM(cfg, w)
    torch.manual_seed(1)
    lens = [12, 5]
    seqs = [torch.randint(0, 100, (n,)) for n in lens]
    ids = torch.cat(seqs)
    pos = torch.cat([torch.arange(n) for n in lens])
    cu = torch.tensor([0, 12, 17], dtype=torch.int32)
    kv = m.allocate_kv_cache(16, 4)
    out = m(StepInput("prefill", ids, pos, torch.arange(17), cu_seqlens=cu, max_seqlen=12,
                      last_idx=torch.tensor([11, 16])), kv)
    for i, s in enumerate(seqs):
        with torch.no_grad():
            ref = hf(s[None]).logits[0, -1]
        assert (out[i, :cfg.vocab_size] - ref).abs().max() < 1e-4


@pytest.mark.parametrize("name", FAMILIES)
def test_greedy_decode_matches_hf(ckpts, name):
    d, hf = ckpts[name]
    cfg, w = _load(d)
    eng = LLMEngine(DecoderLM(cfg, w), max_num_seqs=4, block_size=4, num_blocks=64)
    torch.manual_seed(2)
    prompts = [torch.randint(0, 100, (n,)) for n in (9, 3, 14)]
    outs = eng.generate([p.tolist() for p in prompts], SamplingParams(max_new_tokens=10, is_greedy=True,
                                                                      ignore_eos=True))
    for p, o in zip(prompts, outs):
        with torch.no_grad():
            ref = hf.generate(p[None], max_new_tokens=10, do_sample=False, pad_token_id=0,
                              eos_token_id=None)[0, len(p):].tolist()
        assert o == ref


def test_preemption_keeps_results(ckpts):
    d, _ = ckpts["llama"]
    cfg, w = _load(d)
    m = DecoderLM(cfg, w)
    prompts = [[(7 * i + j) % 100 for j in range(10 + i)] for i in range(6)]
    sp = SamplingParams(max_new_tokens=20, is_greedy=True, ignore_eos=True)
    big = LLMEngine(m, max_num_seqs=8, block_size=4, num_blocks=200).generate(prompts, sp)
    small_eng = LLMEngine(m, max_num_seqs=8, block_size=4, num_blocks=24)  # forces preemption
    small = small_eng.generate(prompts, sp)
    assert small == big
    assert small_eng.stats["preemptions"] > 0


def test_presets_and_params():
    for n in preset_names():
        cfg = get_preset(n)
        assert cfg.head_dim * cfg.num_heads == cfg.hidden_size or cfg.model_type == "llama"
    c = get_preset("llama2-7b")
    assert abs(c.num_params() - 6.74e9) / 6.74e9 < 0.01
    c = get_preset("llama2-70b")
    assert abs(c.num_params() - 68.98e9) / 68.98e9 < 0.01
    p = shard_plan(get_preset("llama2-70b"), 8, 3)
    assert (p.nh_l, p.nkv_l, p.kv_start) == (8, 1, 3)
    p = shard_plan(get_preset("santacoder"), 4, 2)
    assert (p.nh_l, p.nkv_l, p.kv_start) == (4, 1, 0)
    p = shard_plan(get_preset("gpt2"), 4, 1)
    assert p.vocab_padded % 64 == 0 and p.vocab_padded >= 50257


def test_random_weights_shapes():
    cfg = get_preset("tiny-llama")
    w = random_weights(cfg, tp=2, rank=1, dtype=torch.float32)
    plan = shard_plan(cfg, 2, 1)
    L = w.layers[0]
    assert L.qkv.w.shape == ((plan.nh_l + 2 * plan.nkv_l) * cfg.head_dim, cfg.hidden_size)
    assert L.up.w.shape == (2 * plan.F_l, cfg.hidden_size) and L.up.glu
    assert L.o.b is None and w.head.w.shape[0] == plan.v_l


@pytest.mark.parametrize("name", ["llama", "gpt2", "gptj"])
def test_shard_cache_roundtrip(tmp_path, name):
    """Per-rank shard cache: the second build mmaps the cached shard, same logits."""
    from llmss_amd.engine import build_model
    from llmss_amd.models.decoder import StepInput

    d = str(tmp_path / name)
    save_hf_model(name, d, vocab=101)
    cache = str(tmp_path / "cache")
    m1 = build_model(d, None, "fp32", "cpu", shard_cache=cache)
    files = [os.path.join(r, f) for r, _, fs in os.walk(cache) for f in fs]
    assert len(files) == 1 and files[0].endswith("tp1-r0-float32.safetensors")
    m2 = build_model(d, None, "fp32", "cpu", shard_cache=cache)
    ids = torch.tensor([5, 17, 3, 99, 42])
    inp = StepInput(kind="prefill", input_ids=ids, positions=torch.arange(5), slots=None,
                    cu_seqlens=torch.tensor([0, 5], dtype=torch.int32), max_seqlen=5,
                    last_idx=torch.tensor([4]))
    kv1, kv2 = m1.allocate_kv_cache(4, 4), m2.allocate_kv_cache(4, 4)
    assert torch.equal(m1(inp, kv1), m2(inp, kv2))


@pytest.mark.parametrize("tp,rank", [(1, 0), (2, 1)])
def test_tied_head_shares_the_embedding_table(tp, rank):
    cfg = get_preset("gpt2", num_layers=1)
    assert cfg.tie_word_embeddings
    w = random_weights(cfg, tp=tp, rank=rank, dtype=torch.float32)
    plan = shard_plan(cfg, tp, rank)
    assert w.head.w.untyped_storage().data_ptr() == w.wte.untyped_storage().data_ptr()
    lo = rank * plan.v_l
    n = min(cfg.vocab_size, lo + plan.v_l) - lo
    assert torch.equal(w.head.w[:n], w.wte[lo:lo + n]) and w.head.w[n:].abs().sum() == 0
    table = plan.vocab_padded * cfg.hidden_size * 4
    assert w.nbytes() < table + sum(t.numel() * 4 for L in w.layers for t in (L.qkv.w, L.o.w, L.up.w, L.down.w)) * 1.01 \
        + (w.wpe.numel() * 4) + 10 * cfg.hidden_size * 4 * 8


def test_rope_interleave_matches_checkpoint_order(ckpts, monkeypatch, tmp_path):
    """neox RoPE models load with q / k head dims interleaved (gptj-form rotation, fusable into the QKV
    GEMM epilogue): same logits as the checkpoint order; the shard cache keeps the flag."""
    from llmss_amd.models.weights import load_shard, save_shard

    d, _ = ckpts["llama"]
    cfg, w_il = _load(d)
    import llmss_amd.models.weights as W

    monkeypatch.setattr(W, "ROPE_INTERLEAVE", False)
    _, w_ck = _load(d)
    monkeypatch.setattr(W, "ROPE_INTERLEAVE", True)
    assert w_il.rope_interleaved and not w_ck.rope_interleaved
    assert DecoderLM(cfg, w_il).cfg.rope_style == "gptj" and DecoderLM(cfg, w_ck).cfg.rope_style == "neox"
    ids = torch.randint(0, 100, (13,))
    outs = []
    for w in (w_il, w_ck):
        m = DecoderLM(cfg, w)
        kv = m.allocate_kv_cache(8, 4)
        outs.append(m(StepInput("prefill", ids, torch.arange(13), torch.arange(13),
                                cu_seqlens=torch.tensor([0, 13], dtype=torch.int32), max_seqlen=13,
                                last_idx=torch.tensor([12])), kv))
    assert (outs[0] - outs[1]).abs().max() < 1e-4
    p = str(tmp_path / "shard.safetensors")
    save_shard(w_il, p)
    assert load_shard(cfg, p, "cpu", torch.float32).rope_interleaved
