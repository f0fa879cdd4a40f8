"""LM cross-entropy kernel (csrc/loss.hip) against torch's fp32 CrossEntropyLoss, and the
façade's ``labels=`` loss on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("T,V,Vp", [(7, 50257, 50304), (33, 32000, 32000), (5, 101, 112), (4, 13, 13)])
def test_ce_rows_match_torch(dtype, T, V, Vp):
    from llmss_amd import ops
    from llmss_amd.ops import hip as H

    torch.manual_seed(0)
    x = (torch.randn(T, Vp, device="cuda") * 4).to(dtype)
    lab = torch.randint(0, V, (T,), device="cuda")
    lab[1] = -1
    ref = torch.nn.functional.cross_entropy(x[:, :V].float(), lab.clamp(min=0), reduction="none")
    ref[1] = 0
    if Vp % 8 == 0:
        got = H.ce_loss_rows(x, lab, V)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    # shifted, mean over non-ignored labels, on a vocab-trimmed [B, S, Vp][..., :V] view
    xb = x.view(1, T, Vp)[..., :V]
    labels = torch.randint(0, V, (1, T), device="cuda")
    labels[0, 2] = -100
    want = torch.nn.functional.cross_entropy(xb[0, :-1].float(), labels[0, 1:], ignore_index=-100)
    torch.testing.assert_close(ops.cross_entropy(xb, labels), want, rtol=1e-4, atol=1e-4)


def test_facade_loss_on_gpu(tmp_path):
    from transformers import AutoConfig, GPT2Config, GPT2LMHeadModel

    from llmss.server.models.custom_modeling import MODEL_REGISTRY
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    torch.manual_seed(0)
    hf = GPT2LMHeadModel(GPT2Config(n_embd=256, n_layer=2, n_head=4, n_positions=128, vocab_size=1000)).eval()
    hf.save_pretrained(str(tmp_path), safe_serialization=True)
    cfg = AutoConfig.from_pretrained(str(tmp_path))
    m = MODEL_REGISTRY["gpt2"](cfg, Weights(weight_files(str(tmp_path)), torch.device("cuda"), torch.bfloat16, None))
    ids = torch.randint(0, 1000, (2, 24))
    out = m(ids.cuda(), labels=ids.cuda())
    with torch.no_grad():
        ref = hf(ids, labels=ids).loss
    assert abs(float(out.loss) - float(ref)) < 0.05 * float(ref)
