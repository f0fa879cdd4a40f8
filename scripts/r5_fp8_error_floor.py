"""Round 5: the error floor of e4m3 weight quantisation on tests/test_hf_parity_gpu.py::test_fp8_llama_end_to_end_vs_bf16
(fp32 HF Llama, weights fake-quantised per output channel or per K-block, lm_head kept; CPU only)."""
import torch, sys
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT + "/tests"); sys.path.insert(0, ROOT)
from test_hf_parity_gpu import _hf, _prompts, VOCAB
hf = _hf("llama").eval().float()
ps = _prompts()
def logits(model):
    outs = []
    with torch.no_grad():
        for p in ps:
            outs.append(model(torch.tensor([p])).logits[0, :, :VOCAB])
    return torch.cat(outs)
lb = logits(hf)
def q_e4m3_rows(w, blk=None):
    if blk:
        N, K = w.shape
        wb = w.view(N, K // blk, blk)
        s = wb.abs().amax(-1, keepdim=True).clamp_min(1e-12) / 448
        return ((wb / s).to(torch.float8_e4m3fn).float() * s).view(N, K)
    s = w.abs().amax(1, keepdim=True).clamp_min(1e-12) / 448
    return (w / s).to(torch.float8_e4m3fn).float() * s
import copy
for blk in (None, 128, 32):
    m = copy.deepcopy(hf)
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Linear) and "lm_head" not in name:
            mod.weight.data = q_e4m3_rows(mod.weight.data, blk)
    lf = logits(m)
    err = (lb - lf).abs().max() / lb.abs().max()
    cos = torch.nn.functional.cosine_similarity(lb, lf, dim=-1).min()
    print("block", blk, "err", float(err), "cos", float(cos))
