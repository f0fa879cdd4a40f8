"""Lane-level CPU emulation of the gfx950 weight-streaming GEMM (csrc/gemm.hip, gemm_stream_kernel).

The emulator re-derives every address the kernel computes - the global_load_lds staging of X into
the XOR-swizzled LDS image, the per-lane W loads, the A/B fragment reads and the
mfma_f32_16x16x32_bf16 operand/result lane maps (CDNA guide §3) - and checks (a) every global
read is in bounds and (b) the result equals X @ W^T. It catches indexing bugs without a GPU.
"""
import numpy as np
import pytest


def mfma_16x16x32(a_lanes, b_lanes, acc):
    """a_lanes/b_lanes: [64, 8] per-lane fragments; acc: [64, 4]. Lane l: A[l&15][8(l>>4)+j],
    B[8(l>>4)+j][l&15]; C/D: col = l&15, row = 4(l>>4) + i."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for l in range(64):
        A[l & 15, 8 * (l >> 4):8 * (l >> 4) + 8] = a_lanes[l]
        B[8 * (l >> 4):8 * (l >> 4) + 8, l & 15] = b_lanes[l]
    C = A @ B
    out = acc.copy()
    for l in range(64):
        for i in range(4):
            out[l, i] += C[4 * (l >> 4) + i, l & 15]
    return out


def emulate_stream(X, W, MT, NT, KC, splitk):
    M, K = X.shape
    N = W.shape[0]
    ROWS, RB = MT * 16, KC * 2
    XBYTES = ROWS * RB
    assert XBYTES % 4096 == 0
    XINST = XBYTES // 1024 // 4
    SW = min(KC // 8 - 1, 15)
    NG = KC // 64
    nck = (K + KC - 1) // KC
    Y = np.zeros((M, N))
    part = np.zeros((splitk, M, N))
    nbx = (N + 64 * NT - 1) // (64 * NT)
    for bx in range(nbx):
        for split in range(splitk):
            cb, ce = nck * split // splitk, nck * (split + 1) // splitk
            accs = [[[np.zeros((64, 4)) for _ in range(NT)] for _ in range(MT)] for _ in range(4)]
            for c in range(cb, ce):
                kc0 = c * KC
                # ---- stage X (all 4 waves): LDS byte image as element array of RB/2 per row
                xbuf = np.zeros((ROWS, KC))
                for w in range(4):
                    for i in range(XINST):
                        inst = i * 4 + w
                        for lane in range(64):
                            o = inst * 1024 + lane * 16
                            row, pc = o // RB, (o % RB) >> 4
                            gc = pc ^ (row & SW)
                            k = min(kc0 + gc * 8, K - 8)
                            gr = min(row, M - 1)
                            assert 0 <= k and k + 8 <= K and 0 <= gr < M
                            xbuf[row, pc * 8:pc * 8 + 8] = X[gr, k:k + 8]
                tail = (K % KC != 0) and c == nck - 1
                for w in range(4):
                    n0 = bx * 64 * NT + w * 16 * NT
                    for q in range(NG):
                        for s in range(2):
                            b_l = [np.zeros((64, 8)) for _ in range(NT)]
                            for nt in range(NT):
                                for l in range(64):
                                    li, g = l & 15, l >> 4
                                    k = kc0 + 64 * q + 16 * g
                                    ok = (not tail) or k < K
                                    kk = k if k < K else 0
                                    n = min(n0 + nt * 16 + li, N - 1)
                                    assert kk + 16 <= K
                                    seg = W[n, kk:kk + 16]
                                    b_l[nt][l] = seg[8 * s:8 * s + 8] if ok else 0
                            for mt in range(MT):
                                a_l = np.zeros((64, 8))
                                for l in range(64):
                                    li, g = l & 15, l >> 4
                                    r = mt * 16 + li
                                    cc = 8 * q + 2 * g + s
                                    ok = (not tail) or (kc0 + 64 * q + 16 * g < K)
                                    p = cc ^ (r & SW)
                                    a_l[l] = xbuf[r, p * 8:p * 8 + 8] if ok else 0
                                for nt in range(NT):
                                    accs[w][mt][nt] = mfma_16x16x32(a_l, b_l[nt], accs[w][mt][nt])
            for w in range(4):
                n0 = bx * 64 * NT + w * 16 * NT
                for mt in range(MT):
                    for nt in range(NT):
                        for l in range(64):
                            li, g = l & 15, l >> 4
                            for i in range(4):
                                m, n = mt * 16 + 4 * g + i, n0 + nt * 16 + li
                                if m < M and n < N:
                                    part[split, m, n] = accs[w][mt][nt][l, i]
    return part.sum(0)


@pytest.mark.parametrize("M,N,K,MT,NT,KC,S", [
    (5, 128, 512, 1, 1, 256, 1),
    (16, 200, 384, 1, 2, 256, 2),   # N and K tails, split-K
    (33, 128, 256, 4, 1, 256, 1),
    (7, 256, 160, 1, 4, 128, 1),    # K < KC
    (70, 130, 256, 8, 2, 64, 2),
])
def test_stream_gemm_emulation(M, N, K, MT, NT, KC, S):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((M, K))
    W = rng.standard_normal((N, K))
    Y = emulate_stream(X, W, MT, NT, KC, S)
    np.testing.assert_allclose(Y, X @ W.T, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("N,K", [(16, 64), (48, 100), (1536, 4096), (32, 1376)])
def test_packed_weight_layout(N, K):
    """pack_weight: 16-row x 64-k panels, contiguous in k-block order; element (n, k) sits at
    ((n // 16) * K64 + k // 64) * 1024 + (n % 16) * 64 + k % 64; unpack inverts; the reference linear
    accepts the packed form."""
    import torch

    from llmss_amd.ops import reference as R

    g = torch.Generator().manual_seed(N + K)
    w = torch.randn(N, K, generator=g)
    wp = R.pack_weight(w)
    k64 = -(-K // 64)
    assert wp.shape == (N // 16, k64, 16, 64) and wp.is_contiguous()
    flat = wp.reshape(-1)
    for n, k in [(0, 0), (N - 1, K - 1), (N // 2, K // 3), (min(17, N - 1), min(65, K - 1))]:
        assert flat[((n // 16) * k64 + k // 64) * 1024 + (n % 16) * 64 + k % 64] == w[n, k]
    if K % 64:
        assert wp[:, -1, :, K % 64:].abs().sum() == 0  # zero k padding
    assert torch.equal(R.unpack_weight(wp, K), w)
    x = torch.randn(5, K, generator=g)
    assert torch.allclose(R.linear(x, wp), R.linear(x, w))
    with pytest.raises(ValueError):
        R.pack_weight(torch.zeros(24, 64))
