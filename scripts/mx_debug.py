"""Debug aid for the MX-fp8 down-projection path (gemm_mid MXA): isolates the scale handling from the data path."""
import torch

from llmss_amd.ops import hip as H
from llmss_amd.ops import reference as R

dev = torch.device("cuda", 0)
torch.manual_seed(0)
M, F, N = 128, 256, 128
q = torch.randint(0, 120, (M, F), dtype=torch.uint8)  # positive e4m3 values
wd = (torch.randn(N, F) * F ** -0.5).to(torch.bfloat16)
qd, sd = R.quant_fp8_rows(wd)
qd_g, sd_g = qd.to(dev), sd.to(dev)
for label, s in [("unit scales", torch.full((M, F // 32), 127, dtype=torch.uint8)),
                 ("per-row scale", (127 + torch.arange(M) % 4).to(torch.uint8)[:, None].repeat(1, F // 32)),
                 ("per-block scale", (127 + torch.arange(F // 32) % 4).to(torch.uint8)[None, :].repeat(M, 1)),
                 ("random", torch.randint(120, 134, (M, F // 32), dtype=torch.uint8))]:
    ref = R.linear(R.dequant_mx_fp8(q, s), qd, None, w_scale=sd).float()
    for tile in (8, 11, 14):
        y = H.linear_w8a8(H.MxAct(q.to(dev), s.to(dev).contiguous()), qd_g, sd_g, None, tile=tile, depth=3, split=1)
        e = ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item()
        print(f"{label:16s} tile {tile:2d}: max rel err {e:.4f}", flush=True)
