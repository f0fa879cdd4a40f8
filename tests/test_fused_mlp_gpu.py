"""Persistent fused MLP block (csrc/fused_mlp.hip): add + norm -> up (+ SwiGLU / GELU) -> down in ONE launch with
in-launch hand-offs, vs the fp32 PyTorch oracle of the same three ops (ops/reference.py add_norm / linear), for
RMSNorm + SwiGLU (Llama) and LayerNorm + GELU with biases (GPT-2 / BigCode), with the o-projection given as
split-K slabs + bias or as bf16 rows; repeated launches (self-resetting counters) and HIP-graph replay; and a
decode engine with the fused block generating the tokens of the unfused one."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(M, H, F, glu, ln, slabs, seed=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    bf = torch.bfloat16

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, device="cuda", generator=g) * s)

    N1 = 2 * F if glu else F
    wu = rnd(N1, H, s=H ** -0.5).to(bf)
    wd = rnd(H, F, s=F ** -0.5).to(bf)
    nw = (1 + 0.1 * rnd(H)).to(bf)
    nb = (0.1 * rnd(H)).to(bf) if ln else None
    bu = (0.1 * rnd(N1)).to(bf) if ln else None
    bd = (0.1 * rnd(H)).to(bf) if ln else None
    resid = rnd(M, H).to(bf)
    if slabs:
        from llmss_amd.ops.hip import PartialSum

        buf = rnd(slabs * M * H, s=0.5)
        ob = (0.1 * rnd(H)).to(bf) if ln else None
        delta = PartialSum(buf, slabs, M, H, ob, resid.device)
        dref = buf.view(slabs, M, H).sum(0) + (ob.float() if ob is not None else 0)
        dref = dref.to(bf)
    else:
        delta = rnd(M, H).to(bf)
        dref = delta
    return dict(delta=delta, dref=dref, resid=resid, nw=nw, nb=nb, wu=wu, bu=bu, wd=wd, bd=bd, glu=glu, ln=ln)


def _ref(c, act):
    from llmss_amd.ops import reference as R

    y, r = R.add_norm(c["dref"], c["nw"], c["nb"], 1e-5, not c["ln"], c["resid"])
    h = R.linear(y, c["wu"], c["bu"], act, c["glu"])
    out = h.float() @ c["wd"].float().t()
    if c["bd"] is not None:
        out = out + c["bd"].float()
    return r, out


def _run(c, act):
    from llmss_amd.ops import hip as Hh

    resid = c["resid"].clone()
    p = Hh.fused_mlp(c["delta"], resid, c["nw"], c["nb"], 1e-5, not c["ln"], c["wu"], c["bu"], c["wd"], c["bd"],
                     act, c["glu"])
    assert p is not None
    out = p.buf[:p.S * p.M * p.N].view(p.S, p.M, p.N).sum(0)
    if p.bias is not None:
        out = out + p.bias.float()
    return resid, out


@pytest.mark.parametrize("M", [1, 7, 64])
@pytest.mark.parametrize("H,F,glu,ln,act,slabs", [(4096, 11008, True, False, "none", 4),  # Llama-2-7B
                                                  (1600, 6400, False, True, "gelu_tanh", 0),  # GPT-2-XL
                                                  (512, 1024, True, False, "none", 0),
                                                  (768, 3072, False, True, "gelu_tanh", 3)])
def test_fused_mlp_matches_reference(M, H, F, glu, ln, act, slabs):
    from llmss_amd.ops import hip as Hh

    if Hh.fused_mlp_plan(M, H, 2 * F if glu else F, F, glu) is None:
        pytest.skip("no fused plan for this shape on this device")
    c = _case(M, H, F, glu, ln, slabs)
    r_ref, o_ref = _ref(c, act)
    for _ in range(3):  # repeated launches: the counters must have reset themselves
        r, o = _run(c, act)
        torch.cuda.synchronize()
        assert torch.equal(r, r_ref)  # the residual add is exact (one bf16 rounding, as add_norm)
        err = (o - o_ref).abs().max() / o_ref.abs().max()
        assert err < 2e-2, float(err)
    assert not Hh.fused_mlp_error(torch.device("cuda", torch.cuda.current_device()))


def test_fused_mlp_graph_replay():
    from llmss_amd.ops import hip as Hh

    c = _case(64, 1600, 6400, False, True, 0, seed=3)
    r_ref, o_ref = _ref(c, "gelu_tanh")
    resid = c["resid"].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        Hh.fused_mlp(c["delta"], resid.clone(), c["nw"], c["nb"], 1e-5, False, c["wu"], c["bu"], c["wd"], c["bd"],
                     "gelu_tanh", False)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, capture_error_mode="thread_local"):
        p = Hh.fused_mlp(c["delta"], resid, c["nw"], c["nb"], 1e-5, False, c["wu"], c["bu"], c["wd"], c["bd"],
                         "gelu_tanh", False)
    for _ in range(4):
        resid.copy_(c["resid"])
        gr.replay()
        torch.cuda.synchronize()
        out = p.buf[:p.S * p.M * p.N].view(p.S, p.M, p.N).sum(0) + p.bias.float()
        assert torch.equal(resid, r_ref)
        assert (out - o_ref).abs().max() / o_ref.abs().max() < 2e-2


@pytest.mark.parametrize("preset", ["tiny-llama", "tiny-gpt2"])
def test_engine_fused_mlp_decode_matches_unfused(preset, monkeypatch):
    """Greedy decode with every bucket's MLP block fused (LLMSS_FUSED_MLP=1, decode graphs) == unfused."""
    from llmss_amd.engine import LLMEngine, SamplingParams
    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights

    cfg = get_preset(preset, hidden_size=256, num_heads=4, head_dim=64, intermediate_size=512 if preset == "tiny-llama"
                     else 1024, max_position_embeddings=256,
                     **({"num_kv_heads": 2, "rotary_dim": 64} if preset == "tiny-llama" else {"num_kv_heads": 4}))
    w = random_weights(cfg, device="cuda", dtype=torch.bfloat16, seed=11, std=0.05)
    prompts = [[(5 * i + 3 * j) % cfg.vocab_size for j in range(4 + 3 * i)] for i in range(6)]
    sp = SamplingParams(max_new_tokens=16, is_greedy=True, ignore_eos=True)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("LLMSS_FUSED_MLP", mode)
        m = DecoderLM(cfg, w)
        e = LLMEngine(m, max_num_seqs=8, block_size=16, use_graphs=True, autotune=False)
        assert bool(m.fused_mlp_rows) == (mode == "1")
        outs.append(e.generate(prompts, sp))
        del e
    assert outs[0] == outs[1]
