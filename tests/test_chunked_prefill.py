"""Chunked prefill and mixed prefill+decode steps: a prompt cut into chunks that attend
their cached prefix through the paged cache, decodes riding along with prompt chunks, and requests
arriving while others decode must give exactly the tokens of whole-prompt prefill (fp32 on CPU).

The GPU half checks the paged extend-attention kernel against the PyTorch oracle (prefix + causal
chunk, MHA/GQA/MQA, D = 64/128/256) and the engine's chunked generation against whole prompts."""
import pytest
import torch

from helpers import FAMILIES, save_hf_model


@pytest.fixture(scope="module")
def ckpts(tmp_path_factory):
    root = tmp_path_factory.mktemp("chunk")
    out = {}
    for name in FAMILIES:
        d = str(root / name)
        save_hf_model(name, d, vocab=101)
        out[name] = d
    return out


def _prompts():
    return [[(5 * i + 3 * j) % 100 for j in range(7 + 9 * i)] for i in range(4)]  # 7, 16, 25, 34 tokens


def _engine(d, budget, dev="cpu", dtype="fp32", **kw):
    from llmss_amd.engine import LLMEngine, build_model

    m = build_model(d, None, dtype, dev)
    return LLMEngine(m, max_num_seqs=4, max_batched_tokens=budget, block_size=4, num_blocks=128, **kw)


@pytest.mark.parametrize("name", FAMILIES)
def test_chunked_equals_whole_prompt(ckpts, name):
    from llmss_amd.engine import SamplingParams

    sp = SamplingParams(max_new_tokens=6, is_greedy=True, ignore_eos=True)
    ref = _engine(ckpts[name], 256).generate(_prompts(), sp)
    eng = _engine(ckpts[name], 8)  # every prompt > 8 tokens is split; decodes mix with chunks
    got = eng.generate(_prompts(), sp)
    assert got == ref
    assert eng.stats["mixed_decode_tokens"] > 0  # some steps carried decode tokens and a chunk
    assert eng.stats["prefill_steps"] >= 34 // 8


def test_arrivals_during_decode(ckpts):
    """Requests added while others are decoding join as chunks of mixed steps."""
    from llmss_amd.engine import SamplingParams

    sp = SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True)
    ps = _prompts()
    ref = _engine(ckpts["llama"], 256).generate(ps, sp)
    eng = _engine(ckpts["llama"], 12)
    rid = {eng.add_request(ps[0], sp): 0}
    pending = list(range(1, 4))
    steps = 0
    while eng.has_unfinished() or pending:
        if pending and steps % 3 == 2:
            i = pending.pop(0)
            rid[eng.add_request(ps[i], sp)] = i
        eng.step()
        steps += 1
    got = {rid[r.id]: r.output_ids for r in eng.pop_finished()}
    assert [got[i] for i in range(4)] == ref


def test_reference_extend_matches_full_attention():
    """The oracle itself: a chunk over a cached prefix == the tail rows of causal attention."""
    from llmss_amd.ops import reference as R

    torch.manual_seed(0)
    nh, nkv, D, bs, L = 4, 2, 16, 4, 19
    qkv = torch.randn(L, (nh + 2 * nkv) * D)
    full = R.attn_prefill(qkv, [0, L], nh, nkv, D, D ** -0.5)
    kc = torch.zeros(8, nkv, bs, D)
    vc = torch.zeros_like(kc)
    bt = torch.tensor([[5, 2, 7, 0, 1, 3]], dtype=torch.int32)
    slots = torch.tensor([int(bt[0, p // bs]) * bs + p % bs for p in range(L)])
    R.rope_cache(qkv.clone(), torch.arange(L), None, None, kc, vc, slots, nh, nkv, D, 0, "neox", do_rope=False)
    p0 = 11
    got = R.attn_extend(qkv[p0:], kc, vc, bt, torch.tensor([0, L - p0]), torch.tensor([L]), nh, nkv, D, D ** -0.5)
    torch.testing.assert_close(got, full[p0:], rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("nh,nkv,D", [(8, 8, 128), (8, 2, 64), (32, 4, 128), (16, 1, 128), (4, 4, 256), (48, 1, 64)])
def test_extend_kernel_matches_reference(nh, nkv, D):
    from llmss_amd.ops import hip as H
    from llmss_amd.ops import reference as R

    torch.manual_seed(1)
    dev = torch.device("cuda")
    bs, nb = 16, 96
    # (prefix, chunk) per sequence: fresh prompt, long prefix + short chunk, chunk crossing blocks, 1-token chunk
    seqs = [(0, 37), (150, 20), (33, 64), (70, 1), (5, 130)]
    kc = (torch.randn(nb, nkv, bs, D, device=dev) * 0.5).to(torch.bfloat16)
    vc = torch.randn(nb, nkv, bs, D, device=dev).to(torch.bfloat16)
    maxb = max((p + q + bs - 1) // bs for p, q in seqs)
    perm = torch.randperm(nb)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    k = 0
    for i, (p, q) in enumerate(seqs):
        n = (p + q + bs - 1) // bs
        bt[i, :n] = perm[k:k + n].to(torch.int32)
        k += n
    T = sum(q for _, q in seqs)
    qrows = (torch.randn(T, (nh + 2 * nkv) * D, device=dev)).to(torch.bfloat16)
    cu = torch.tensor([0] + torch.tensor([q for _, q in seqs]).cumsum(0).tolist(), dtype=torch.int32)
    ctx = torch.tensor([p + q for p, q in seqs], dtype=torch.int32)
    scale = D ** -0.5
    got = H.attn_extend(qrows, kc, vc, bt.to(dev), cu.to(dev), ctx.to(dev), max(q for _, q in seqs), nh, nkv, D,
                        scale)
    ref = R.attn_extend(qrows.float().cpu(), kc.float().cpu(), vc.float().cpu(), bt, cu, ctx, nh, nkv, D, scale)
    torch.testing.assert_close(got.float().cpu(), ref, rtol=2e-2, atol=2e-2)


def _save_gpu_model(name, path, vocab=101):
    """Tiny checkpoints with GPU-kernel head sizes (D = 64 / 256)."""
    from transformers import (GPTBigCodeConfig, GPTBigCodeForCausalLM, GPTJConfig, GPTJForCausalLM, LlamaConfig,
                              LlamaForCausalLM)

    torch.manual_seed(0)
    kw = dict(vocab_size=vocab, bos_token_id=vocab - 1, eos_token_id=vocab - 1)
    if name == "llama":
        m = LlamaForCausalLM(LlamaConfig(hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                         num_key_value_heads=2, intermediate_size=512, max_position_embeddings=256,
                                         initializer_range=0.1, **kw))
    elif name == "gptj":
        m = GPTJForCausalLM(GPTJConfig(n_embd=512, n_layer=2, n_head=2, n_positions=256, rotary_dim=64,
                                       initializer_range=0.1, **kw))
    else:
        m = GPTBigCodeForCausalLM(GPTBigCodeConfig(n_embd=256, n_layer=2, n_head=4, n_positions=256, multi_query=True,
                                                   initializer_range=0.1, **kw))
    m.eval().save_pretrained(path, safe_serialization=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["llama", "gptj", "bigcode"])
def test_gpu_chunked_engine_matches_whole_prompt(tmp_path, name):
    from llmss_amd.engine import SamplingParams

    d = str(tmp_path / name)
    _save_gpu_model(name, d)
    dev = torch.device("cuda", 0)
    sp = SamplingParams(max_new_tokens=6, is_greedy=True, ignore_eos=True)
    ref_eng = _engine(d, 256, dev, "bf16", use_graphs=False, autotune=False)
    ref = ref_eng.generate(_prompts(), sp)
    eng = _engine(d, 8, dev, "bf16", use_graphs=False, autotune=False)
    got = eng.generate(_prompts(), sp)
    assert eng.stats["mixed_decode_tokens"] > 0
    # bf16: the chunked path adds the same terms in another order, so a greedy pick may flip where the
    # fp32 model itself has a near tie (the top-2 margin under 0.1 on these ~3-logit tiny models; a
    # measured case: 3.204 vs 3.157). Every token must match up to such a tie; after a tie the
    # sequences are conditioned on different tokens and comparison stops.
    from transformers import AutoModelForCausalLM

    hf = AutoModelForCausalLM.from_pretrained(d).float().eval()
    compared = 0
    for p, g, r in zip(_prompts(), got, ref):
        for k, (a, b) in enumerate(zip(g, r)):
            if a == b:
                compared += 1
                continue
            with torch.no_grad():
                top2 = hf(torch.tensor([p + r[:k]])).logits[0, -1].topk(2).values
            assert float(top2[0] - top2[1]) < 0.1, ("chunked and whole-prompt runs differ at a clear margin",
                                                    name, k, top2.tolist(), got, ref)
            break
    assert compared >= 0.6 * sum(len(x) for x in ref), (compared, got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("nh,D", [(8, 128), (4, 64), (16, 128), (2, 256)])
def test_extend_kernel_fp8_twin_equals_the_quant_launch(nh, D):
    """One kv head per rank (Llama-2-70B at TP=8: 8 query heads): the extend kernel's fused per-token fp8 twin of its
    output equals quant_fp8_rows_ld of that output bit for bit (same absmax / 448 scale, same clamped conversion),
    for decode rows and multi-token chunks, and the bf16 output is unchanged; the twin is registered for the W8A8
    o-projection that consumes the tensor next."""
    from llmss_amd.ops import hip as H

    torch.manual_seed(3)
    dev = torch.device("cuda")
    nkv, bs, nb = 1, 16, 96
    seqs = [(0, 37), (150, 20), (33, 64), (70, 1), (5, 130), (16, 1), (200, 1)]
    kc = (torch.randn(nb, nkv, bs, D, device=dev) * 0.5).to(torch.bfloat16)
    vc = torch.randn(nb, nkv, bs, D, device=dev).to(torch.bfloat16)
    maxb = max((p + q + bs - 1) // bs for p, q in seqs)
    perm = torch.randperm(nb)
    bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
    k = 0
    for i, (p, q) in enumerate(seqs):
        n = (p + q + bs - 1) // bs
        bt[i, :n] = perm[k:k + n].to(torch.int32)
        k += n
    T = sum(q for _, q in seqs)
    qrows = (torch.randn(T, (nh + 2 * nkv) * D, device=dev)).to(torch.bfloat16)
    cu = torch.tensor([0] + torch.tensor([q for _, q in seqs]).cumsum(0).tolist(), dtype=torch.int32, device=dev)
    ctx = torch.tensor([p + q for p, q in seqs], dtype=torch.int32, device=dev)
    bt = bt.to(dev)
    mq = max(q for _, q in seqs)
    assert H.extend_fp8_twin_ok(nh, nkv)
    plain = H.attn_extend(qrows, kc, vc, bt, cu, ctx, mq, nh, nkv, D, D ** -0.5)
    got = H.attn_extend(qrows, kc, vc, bt, cu, ctx, mq, nh, nkv, D, D ** -0.5, fp8_out=True)
    assert torch.equal(got, plain)
    tq, ts = H._prequant_of(got)
    K = nh * D
    rq = torch.empty(T, K, dtype=torch.uint8, device=dev)
    rs = torch.empty(T, dtype=torch.float32, device=dev)
    H.lib().quant_fp8_rows_ld(got.data_ptr(), got.stride(0), rq.data_ptr(), rs.data_ptr(), T, K, H._stream())
    torch.cuda.synchronize()
    assert torch.equal(ts, rs)
    assert torch.equal(tq, rq)
    # heads of a row spread over workgroups / waves: no fused twin
    assert not H.extend_fp8_twin_ok(8, 2) and not H.extend_fp8_twin_ok(32, 1) and not H.extend_fp8_twin_ok(12, 1)
