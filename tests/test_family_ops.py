"""Reference module-level helpers and per-family classes at the reference import paths
(``llmss.server.models.custom_modeling.{gptj_modeling, gpt_bigcode_modeling}``), checked against the same-named
functions of HF transformers' GPT-J / GPTBigCode modules, which the reference's versions match."""
import pytest
import torch

from helpers import save_hf_model


def test_gptj_rotary_helpers_match_hf():
    import transformers.models.gptj.modeling_gptj as hf
    from llmss.server.models.custom_modeling import gptj_modeling as ours

    for n, d in ((64, 16), (2048, 64)):
        torch.testing.assert_close(ours.create_sinusoidal_positions(n, d), hf.create_sinusoidal_positions(n, d),
                                   rtol=0, atol=2e-4)
    x = torch.randn(2, 5, 3, 16)
    torch.testing.assert_close(ours.rotate_every_two(x), hf.rotate_every_two(x), rtol=0, atol=0)
    table = hf.create_sinusoidal_positions(64, 16)
    pos = torch.randint(0, 64, (2, 5))
    emb = ours.get_embed_positions(table, pos)
    assert emb.shape == (2, 64, 16) and torch.equal(emb[1], table)
    sincos = torch.gather(emb, 1, pos[..., None].expand(-1, -1, 16))
    sin, cos = torch.split(sincos, 8, dim=-1)
    for dt in (torch.float32, torch.bfloat16):
        xt = x.to(dt)
        ref = hf.apply_rotary_pos_emb(xt, sin, cos)
        got = ours.apply_rotary_pos_emb(xt, sin, cos)
        assert got.dtype == ref.dtype
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_bigcode_softmax_helpers_match_hf():
    import transformers.models.gpt_bigcode.modeling_gpt_bigcode as hf
    from llmss.server.models.custom_modeling import gpt_bigcode_modeling as ours

    x = torch.randn(2, 4, 7, 7, dtype=torch.bfloat16)
    mask = torch.tril(torch.ones(7, 7, dtype=torch.bool))[None, None]
    mv = torch.full([], torch.finfo(torch.float32).min)
    torch.testing.assert_close(ours.upcast_softmax(x, 0.3, torch.float32), hf.upcast_softmax(x, 0.3, torch.float32))
    torch.testing.assert_close(ours.upcast_masked_softmax(x, mask, mv, 0.3, torch.float32),
                               hf.upcast_masked_softmax(x, mask, mv, 0.3, torch.float32))
    xf = x.float()
    torch.testing.assert_close(ours.masked_softmax(xf, mask, mv), hf.masked_softmax(xf, mask, mv))


@pytest.mark.parametrize("name,cls", [("gptj", "GPTJForCausalLM"), ("bigcode", "GPTBigCodeForCausalLM")])
def test_family_classes_at_reference_paths(tmp_path, name, cls):
    from transformers import AutoConfig

    import llmss.server.models.custom_modeling as cm
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    d = str(tmp_path / name)
    hf = save_hf_model(name, d)
    config = AutoConfig.from_pretrained(d)
    assert cm.MODEL_REGISTRY[config.model_type] is getattr(cm, cls)
    w = Weights(weight_files(d), torch.device("cpu"), torch.float32, None)
    model = getattr(cm, cls)(config, w).eval()
    ids = torch.randint(0, 100, (2, 7))
    with torch.no_grad():
        ref = hf(ids).logits
    torch.testing.assert_close(model(ids).logits, ref, rtol=1e-4, atol=1e-4)
    other = cm.GPTBigCodeForCausalLM if cls == "GPTJForCausalLM" else cm.GPTJForCausalLM
    with pytest.raises(ValueError, match="model_type"):
        other(config, w)
