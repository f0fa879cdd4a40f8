"""End-to-end GPU parity against HF transformers checkpoints (fp32 HF on CPU as the oracle):
prefill logits and greedy continuations of all five families through the native bf16 kernels, fp8
(W8A16 / W8A8) Llama against its bf16 twin, and generate.py's no-cache (recompute) mode against its
cached mode on the GPU."""
import ast
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

VOCAB = 1000


def _hf(name):
    from transformers import (GPT2Config, GPT2LMHeadModel, GPTBigCodeConfig, GPTBigCodeForCausalLM, GPTJConfig,
                              GPTJForCausalLM, LlamaConfig, LlamaForCausalLM)

    torch.manual_seed(0)
    kw = dict(vocab_size=VOCAB, bos_token_id=VOCAB - 1, eos_token_id=VOCAB - 1)
    if name == "gpt2":
        return GPT2LMHeadModel(GPT2Config(n_embd=256, n_layer=3, n_head=4, n_positions=256, initializer_range=0.05,
                                          **kw))
    if name == "gptj":
        return GPTJForCausalLM(GPTJConfig(n_embd=512, n_layer=2, n_head=2, n_positions=256, rotary_dim=64,
                                          initializer_range=0.05, **kw))
    if name == "bigcode":
        return GPTBigCodeForCausalLM(GPTBigCodeConfig(n_embd=512, n_layer=2, n_head=4, n_positions=256,
                                                      multi_query=True, initializer_range=0.05, **kw))
    if name == "bigcode_mha":
        return GPTBigCodeForCausalLM(GPTBigCodeConfig(n_embd=256, n_layer=2, n_head=4, n_positions=256,
                                                      multi_query=False, initializer_range=0.05, **kw))
    return LlamaForCausalLM(LlamaConfig(hidden_size=512, num_hidden_layers=2, num_attention_heads=4,
                                        num_key_value_heads=2, intermediate_size=1024, max_position_embeddings=256,
                                        initializer_range=0.05, **kw))


def _prompts():
    g = torch.Generator().manual_seed(5)
    return [torch.randint(0, VOCAB - 1, (n,), generator=g).tolist() for n in (9, 31, 64, 17)]


@pytest.mark.parametrize("name", ["gpt2", "gptj", "bigcode", "bigcode_mha", "llama"])
def test_native_bf16_matches_hf(tmp_path, name):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.models.decoder import StepInput

    hf = _hf(name).eval()
    hf.save_pretrained(str(tmp_path), safe_serialization=True)
    dev = torch.device("cuda", 0)
    m = build_model(str(tmp_path), None, "bf16", dev)
    ps = _prompts()
    # all-position prefill logits of the packed batch vs HF per prompt
    ids = torch.tensor([t for p in ps for t in p], device=dev)
    pos = torch.cat([torch.arange(len(p)) for p in ps]).to(dev)
    cu = torch.tensor([0] + torch.tensor([len(p) for p in ps]).cumsum(0).tolist(), dtype=torch.int32, device=dev)
    kv = m.allocate_kv_cache(32, 16)
    inp = StepInput("prefill", ids, pos, torch.full_like(ids, -1), cu_seqlens=cu, max_seqlen=max(map(len, ps)))
    got = m(inp, kv)[:, :VOCAB].float().cpu()
    with torch.no_grad():
        ref = torch.cat([hf(torch.tensor([p])).logits[0] for p in ps])
    scale = ref.abs().max()
    err = (got - ref).abs().max() / scale
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1).min()
    assert err < 3e-2 and cos > 0.999, (name, float(err), float(cos))
    # greedy continuations through the engine (paged decode, HIP graphs) vs HF generate
    eng = LLMEngine(m, max_num_seqs=4, block_size=16, autotune=False)
    out = eng.generate(ps, SamplingParams(max_new_tokens=10, is_greedy=True, ignore_eos=True))
    # margin-aware greedy agreement: every token must match HF's greedy token, except at a position where HF's
    # own top-2 logit margin is within bf16 noise (a few times the measured prefill error): there a flip is a
    # tie-break, and the rest of that sequence is conditioned on a different token, so comparison stops
    noise = max(4 * float(err) * float(scale), 1e-3)
    compared = ties = 0
    for p, o in zip(ps, out):
        with torch.no_grad():
            r = hf.generate(torch.tensor([p]), max_new_tokens=10, do_sample=False, min_new_tokens=10,
                            pad_token_id=0)[0, len(p):].tolist()
            lg = hf(torch.tensor([p + r])).logits[0, len(p) - 1:len(p) + len(r) - 1]
        top2 = lg.topk(2, dim=-1).values
        margin = (top2[:, 0] - top2[:, 1]).tolist()
        for i, (a, b) in enumerate(zip(o, r)):
            if a == b:
                compared += 1
                continue
            assert margin[i] < noise, (name, "greedy token differs at a clear margin", i, margin[i], noise, o, r)
            ties += 1
            break
    assert compared >= 0.75 * 10 * len(ps), (name, compared, ties, out)


def test_fp8_llama_end_to_end_vs_bf16(tmp_path):
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.models.decoder import StepInput

    hf = _hf("llama").eval()
    hf.save_pretrained(str(tmp_path), safe_serialization=True)
    dev = torch.device("cuda", 0)
    ps = _prompts()
    outs = {}
    for fp8 in (False, True):
        m = build_model(str(tmp_path), None, "bf16", dev, fp8=fp8)
        assert (m.w.layers[0].qkv.w.dtype == torch.uint8) == fp8  # e4m3 weight bytes + per-channel scales
        ids = torch.tensor([t for p in ps for t in p], device=dev)
        pos = torch.cat([torch.arange(len(p)) for p in ps]).to(dev)
        cu = torch.tensor([0] + torch.tensor([len(p) for p in ps]).cumsum(0).tolist(), dtype=torch.int32, device=dev)
        inp = StepInput("prefill", ids, pos, torch.full_like(ids, -1), cu_seqlens=cu, max_seqlen=max(map(len, ps)),
                        last_idx=(cu[1:] - 1).long())
        lg = m(inp, m.allocate_kv_cache(32, 16))[:, :VOCAB].float().cpu()
        eng = LLMEngine(m, max_num_seqs=4, block_size=16, autotune=False)
        gen = eng.generate(ps, SamplingParams(max_new_tokens=12, is_greedy=True, ignore_eos=True))
        outs[fp8] = (lg, gen)
        del eng, m
        torch.cuda.empty_cache()
    (lb, gb), (lf, gf) = outs[False], outs[True]
    cos = torch.nn.functional.cosine_similarity(lb, lf, dim=-1).min()
    err = (lb - lf).abs().max() / lb.abs().max()
    print(f"fp8 vs bf16 logits: min cosine {float(cos):.5f}, max err / max |logit| {float(err):.4f}")
    assert cos > 0.99 and err < 0.15, (float(cos), float(err))
    first = sum(a[0] == b[0] for a, b in zip(gb, gf))
    assert first >= 3, (gb, gf)


def test_generate_cli_recompute_mode_on_gpu(tmp_path):
    from helpers import make_tokenizer

    hf = _hf("gpt2")
    hf.save_pretrained(str(tmp_path), safe_serialization=True)
    make_tokenizer(str(tmp_path), 101)  # ids < 101 of the 1000-entry vocabulary
    prompts = ["hello world", "this is a tiny"]
    outs = []
    for cache in ([], ["--use_cache"]):
        r = subprocess.run([sys.executable, "generate.py", "--pretrained_model_path", str(tmp_path), "--prompts",
                            *prompts, "--max_new_tokens", "8", "--is_greedy", "--device", "cuda", *cache],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = r.stdout.strip().splitlines()
        assert lines[0].startswith("elapsed time: ") and lines[1] == f"prompts: {prompts}"
        outs.append(ast.literal_eval(lines[2][len("continuations: "):]))
        assert "cuda" in r.stdout  # the timing line names the device the run used
    assert outs[0] == outs[1]  # recompute (no cache) == paged-cache decode
