"""The MX-fp8 activation format of the W8A8 MLP hand-off (gate/up SwiGLU epilogue -> down projection,
csrc/common.h img_store_rows + csrc/gemm_mid.hip MXA), in the CPU reference (ops/reference.py quant_mx_fp8): the
block scale is the smallest power of two that fits the block under e4m3's 448, the round trip is within half an
e4m3 step, zero blocks stay zero, and blocks far below the row maximum keep their precision."""
import torch

from llmss_amd.ops import reference as R


def test_mx_scale_is_the_smallest_fitting_power_of_two():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(37, 256, generator=g) * torch.logspace(-6, 6, 37)[:, None]
    x[3, 32:64] = 0.0  # an all-zero block
    x[5, 0] = 448.0 * 2.0 ** 3  # exactly 448 * 2^e: e = 3, not 4
    q, s = R.quant_mx_fp8(x)
    assert q.shape == (37, 256) and s.shape == (37, 8) and q.dtype == s.dtype == torch.uint8
    e = s.to(torch.int32) - 127
    amax = x.reshape(37, 8, 32).abs().amax(-1)
    nz = amax > 0
    assert (amax[nz] / torch.ldexp(torch.ones(()), e[nz]) <= 448).all()
    assert (amax[nz] / torch.ldexp(torch.ones(()), e[nz] - 1) > 448).all()  # one step smaller would not fit
    assert e[5, 0] == 3 and e[3, 1] == 0 and (q[3, 32:64] == 0).all()
    y = R.dequant_mx_fp8(q, s)
    assert (y[3, 32:64] == 0).all()
    # e4m3 keeps 3 mantissa bits: |y - x| <= 2^-4 |x| plus the subnormal floor of the block
    floor = torch.ldexp(torch.ones(()), e - 9).repeat_interleave(32, 1)
    assert ((y - x).abs() <= x.abs() * 2.0 ** -4 + floor).all()


def test_mx_keeps_the_blocks_that_per_token_scaling_flushes():
    """Within e4m3's range both scalings keep 3 mantissa bits (same relative error); a row spanning more than that
    range (2^-6 .. 448 normal, subnormals to 2^-9) loses its small blocks to one per-row scale but keeps them under
    per-32 block scales."""
    g = torch.Generator().manual_seed(1)
    x = torch.randn(64, 1024, generator=g) * torch.logspace(-7, 1, 32).repeat_interleave(32)[None, :]
    e_mx = (R.fake_quant_mx_act(x) - x).norm() / x.norm()
    e_tok = (R.fake_quant_fp8_act(x) - x).norm() / x.norm()
    assert e_mx < 1.1 * e_tok  # the large blocks dominate both norms: same precision there
    small = slice(0, 256)  # blocks 10^4 - 10^7 below the row maximum
    rel = lambda f: ((f(x)[:, small] - x[:, small]).norm() / x[:, small].norm()).item()  # noqa: E731
    assert rel(R.fake_quant_mx_act) < 0.05 and rel(R.fake_quant_fp8_act) > 0.5
