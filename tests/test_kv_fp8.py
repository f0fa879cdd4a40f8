"""fp8 paged KV cache (LLMEngine(kv_dtype="fp8") / LLMSS_KV_DTYPE=fp8): each (token, kv head) row is
head_dim e4m3 bytes + a 16-byte tail holding the row's fp32 scale (absmax / 448), written by the rope /
cache kernel and read by decode and extend attention. Oracles: ops/reference.py (kv_rows_quant /
kv_rows_dequant and the paged attention references, which dequantise), fp32 math."""
import math

import pytest
import torch

from helpers import save_hf_model


def test_row_quant_roundtrip_cpu():
    from llmss_amd.ops import reference as R

    torch.manual_seed(0)
    x = torch.randn(7, 3, 128) * torch.tensor([0.01, 1.0, 50.0])[None, :, None]
    rows = R.kv_rows_quant(x)
    assert rows.shape == (7, 3, 128 + 16) and rows.dtype == torch.uint8
    back = R.kv_rows_dequant(rows, 128)
    amax = x.abs().amax(-1, keepdim=True)
    # e4m3: 3 mantissa bits -> half an ulp is <= 1/16 of the value; values below 2^-6 * scale are subnormal
    assert ((back - x).abs() <= x.abs() / 16 + amax / 448 * 2 ** -9 + 1e-12).all()
    assert torch.equal(rows[..., 132:], torch.zeros_like(rows[..., 132:]))
    z = R.kv_rows_quant(torch.zeros(2, 64))  # all-zero rows: scale 1, no NaN
    assert torch.equal(R.kv_rows_dequant(z, 64), torch.zeros(2, 64))


@pytest.mark.parametrize("name", ["llama", "gpt2"])
def test_engine_fp8_kv_cpu(tmp_path, name):
    """CPU plumbing: the engine allocates fp8 rows, and greedy decoding through them stays close to bf16."""
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    d = str(tmp_path / name)
    save_hf_model(name, d, vocab=101)
    prompts = [[(3 * i + 7 * j) % 100 for j in range(5 + 2 * i)] for i in range(3)]
    outs = {}
    for kv in ("bf16", "fp8"):
        m = build_model(d, None, "fp32", "cpu")
        eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64, kv_dtype=kv)
        if kv == "fp8":
            assert eng.kv[0][0].dtype == torch.uint8 and eng.kv[0][0].shape[-1] == m.cfg.head_dim + 16
            assert eng.fingerprint()["kv_fp8"]
        outs[kv] = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    agree = sum(a == b for x, y in zip(outs["bf16"], outs["fp8"]) for a, b in zip(x, y))
    assert agree >= 0.8 * sum(len(x) for x in outs["bf16"]), outs


# ------------------------------------------------------------------------------------------------ GPU
dev = torch.device("cuda")


def _caches(nb, nkv, bs, D):
    from llmss_amd.ops import reference as R

    k = torch.randn(nb, nkv, bs, D) * 0.7
    v = torch.randn(nb, nkv, bs, D)
    return R.kv_rows_quant(k).to(dev), R.kv_rows_quant(v).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("style,D,rot,nh,nkv", [("neox", 128, 128, 8, 2), ("neox", 128, 64, 4, 4), ("gptj", 256, 64, 4, 4),
                                                ("neox", 64, 0, 4, 4)])
def test_rope_cache_writes_fp8_rows(style, D, rot, nh, nkv):
    from llmss_amd.ops import hip as H
    from llmss_amd.ops import reference as R

    torch.manual_seed(0)
    T, bs, nb = 37, 16, 8
    qkv = (torch.randn(T, (nh + 2 * nkv) * D) * 2).to(torch.bfloat16)
    pos = torch.randint(0, 500, (T,))
    cos, sin = R.rope_tables(512, max(rot, 8), 10000.0)
    slots = torch.randperm(nb * bs)[:T]
    slots[3] = -1  # padding row: not cached
    kc = torch.zeros(nb, nkv, bs, D + 16, dtype=torch.uint8)
    vc = torch.zeros_like(kc)
    q_ref = qkv.clone()
    R.rope_cache(q_ref, pos, cos, sin, kc, vc, slots, nh, nkv, D, rot, style, do_rope=rot > 0)
    q_gpu = qkv.to(dev)
    kg, vg = torch.zeros_like(kc, device=dev), torch.zeros_like(vc, device=dev)
    H.rope_cache(q_gpu, pos.to(dev), cos.to(dev), sin.to(dev), kg, vg, slots.to(dev), nh, nkv, D, rot, style,
                 do_rope=rot > 0)
    torch.testing.assert_close(q_gpu.float().cpu(), q_ref.float(), rtol=1e-2, atol=1e-2)
    for got, ref in ((kg.cpu(), kc), (vg.cpu(), vc)):
        assert torch.equal(got[..., D + 4:], ref[..., D + 4:])  # zero tails
        sg, sr = R.kv_rows_dequant(got, D), R.kv_rows_dequant(ref, D)
        scale = ref[..., D:D + 4].contiguous().view(torch.float32)
        # same scale; values within one e4m3 step of the oracle's (rotation arithmetic may round differently)
        torch.testing.assert_close(got[..., D:D + 4].contiguous().view(torch.float32), scale, rtol=1e-2, atol=1e-6)
        assert ((sg - sr).abs() <= sr.abs() / 8 + scale * 2 ** -6).all()


@pytest.mark.gpu
@pytest.mark.parametrize("D,nh,nkv", [(128, 32, 32), (128, 32, 8), (64, 25, 25), (256, 16, 16), (128, 8, 1)])
def test_decode_attention_fp8_rows(D, nh, nkv):
    from llmss_amd.ops import hip as H
    from llmss_amd.ops import reference as R

    torch.manual_seed(0)
    B, bs, maxctx = 6, 16, 300
    maxb = (maxctx + bs - 1) // bs
    nb = B * maxb + 3
    kc, vc = _caches(nb, nkv, bs, D)
    bt = torch.randperm(nb, device=dev)[: B * maxb].view(B, maxb).to(torch.int32)
    ctx = torch.randint(1, maxctx + 1, (B,), device=dev, dtype=torch.int32)
    ctx[0] = maxctx
    q = torch.randn(B, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
    sc = 1 / math.sqrt(D)
    ref = R.attn_decode(q.float().cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), nh, nkv, D, sc)
    try:
        for u in (0, 2, 12):
            H.lib().attn_decode_set_unroll(u)
            for splits in (None, (1, maxb * bs)):
                got = H.attn_decode(q, kc, vc, bt, ctx, nh, nkv, D, sc, maxctx, splits=splits)
                torch.testing.assert_close(got.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    finally:
        H.lib().attn_decode_set_unroll(0)


@pytest.mark.gpu
@pytest.mark.parametrize("nh,nkv,D", [(8, 8, 128), (32, 4, 128), (8, 2, 64), (4, 4, 256)])
def test_extend_attention_fp8_rows(nh, nkv, D):
    from llmss_amd.ops import hip as H
    from llmss_amd.ops import reference as R

    torch.manual_seed(1)
    bs, nb = 16, 96
    seqs = [(0, 37), (150, 20), (33, 64), (70, 1)]
    kc, vc = _caches(nb, nkv, bs, D)
    maxb = max((p + q + bs - 1) // bs for p, q in seqs)
    perm = torch.randperm(nb)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    k = 0
    for i, (p, q) in enumerate(seqs):
        n = (p + q + bs - 1) // bs
        bt[i, :n] = perm[k:k + n].to(torch.int32)
        k += n
    T = sum(q for _, q in seqs)
    qrows = torch.randn(T, (nh + 2 * nkv) * D, device=dev).to(torch.bfloat16)
    cu = torch.tensor([0] + torch.tensor([q for _, q in seqs]).cumsum(0).tolist(), dtype=torch.int32)
    ctx = torch.tensor([p + q for p, q in seqs], dtype=torch.int32)
    scale = D ** -0.5
    got = H.attn_extend(qrows, kc, vc, bt.to(dev), cu.to(dev), ctx.to(dev), max(q for _, q in seqs), nh, nkv, D, scale)
    ref = R.attn_extend(qrows.float().cpu(), kc.cpu(), vc.cpu(), bt, cu, ctx, nh, nkv, D, scale)
    torch.testing.assert_close(got.float().cpu(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_engine_fp8_kv_gpu(tmp_path):
    """Llama (GQA) end to end on the GPU with chunked prefill (prompt chunks read their cached prefix
    through the extend kernel): fp8 rows halve the KV bytes and greedy tokens stay mostly equal to the
    bf16 cache's."""
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    from transformers import LlamaConfig, LlamaForCausalLM

    d = str(tmp_path / "llama")
    torch.manual_seed(0)
    LlamaForCausalLM(LlamaConfig(vocab_size=1000, hidden_size=512, num_hidden_layers=2, num_attention_heads=4,
                                 num_key_value_heads=2, intermediate_size=1024, max_position_embeddings=256,
                                 initializer_range=0.05, bos_token_id=999, eos_token_id=999)).save_pretrained(
        d, safe_serialization=True)
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(0, 999, (n,), generator=g).tolist() for n in (9, 31, 64, 17)]
    outs, blocks = {}, {}
    for kv in ("bf16", "fp8"):
        m = build_model(d, None, "bf16", dev)
        eng = LLMEngine(m, max_num_seqs=4, block_size=16, kv_dtype=kv, autotune=False, prefill_chunk=16)
        outs[kv] = eng.generate(prompts, SamplingParams(max_new_tokens=16, is_greedy=True, ignore_eos=True))
        blocks[kv] = m.kv_bytes_per_block(16)
        del eng, m
        torch.cuda.empty_cache()
    assert blocks["fp8"] * 1.7 < blocks["bf16"]
    agree = sum(a == b for x, y in zip(outs["bf16"], outs["fp8"]) for a, b in zip(x, y))
    assert agree >= 0.6 * sum(len(x) for x in outs["bf16"]), outs
