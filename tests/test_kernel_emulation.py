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


class _RingModel:
    """Program-order model of one wave of a ring schedule (all waves run the same program; a barrier means every
    wave has finished everything before it). Records which stage each LDS slot holds and checks the two ring
    invariants: a fragment read sees a stage that has landed for every wave (a vmcnt wait that covers it, then a
    barrier), and no slot is restaged before every wave's reads of its previous stage have completed (an lgkmcnt
    wait, then a barrier)."""

    def __init__(self, ns):
        self.ns = ns
        self.slot = [None] * ns        # stage held by each slot
        self.issued = []               # stages in issue order
        self.landed = set()            # stages whose loads this wave has waited for
        self.visible = set()           # ... and that a barrier since made visible to every wave
        self.reads = {}                # slot -> "pending" | "done" | "synced" (reads of its current stage)

    def issue(self, stage, slot):
        assert self.reads.get(slot, "synced") == "synced", f"slot {slot} restaged while reads of stage {self.slot[slot]} may be in flight"
        self.slot[slot] = stage
        self.reads[slot] = "synced"
        self.issued.append(stage)

    def vm_wait(self, younger):
        # s_waitcnt vmcnt(younger * LOADS): every stage but the `younger` newest ones has landed
        done = self.issued[:len(self.issued) - younger] if younger else list(self.issued)
        self.landed.update(done)

    def lgkm_wait(self):
        for s, st in self.reads.items():
            if st == "pending":
                self.reads[s] = "done"

    def barrier(self):
        self.lgkm_wait()  # every barrier of the kernel is preceded by lgkmcnt(0)
        self.visible |= self.landed
        for s, st in self.reads.items():
            if st == "done":
                self.reads[s] = "synced"

    def read(self, slot, stage):
        assert self.slot[slot] == stage, f"slot {slot} holds stage {self.slot[slot]}, expected {stage}"
        assert stage in self.visible, f"stage {stage} read before it landed for every wave"
        self.reads[slot] = "pending"


def _ilv_schedule(ns, t0, t1):
    """csrc/gemm_mid.hip gemm_mid_kernel, ILV path: the order of stage issues, waits, barriers and reads."""
    r = _RingModel(ns)
    for j in range(ns - 1):
        if t0 + j < t1:
            r.issue(t0 + j, j)
    r.vm_wait(min(t1 - 1 - t0, ns - 2))
    r.barrier()
    r.read(0, t0)  # first-half fragments of k-step t0
    r.lgkm_wait()
    cur, t = 0, t0
    while t + ns - 1 < t1:  # steady state
        nx = 0 if cur == ns - 1 else cur + 1
        r.read(cur, t)  # second-half fragments (under the first-half MFMAs)
        r.vm_wait(ns - 3)
        r.barrier()
        r.issue(t + ns - 1, ns - 1 if cur == 0 else cur - 1)
        r.read(nx, t + 1)  # next k-step's first half (under the second-half MFMAs)
        r.lgkm_wait()
        cur, t = nx, t + 1
    while t < t1:  # tail: nothing left to stage
        nx = 0 if cur == ns - 1 else cur + 1
        r.read(cur, t)
        if t + 1 < t1:
            r.vm_wait(t1 - 2 - t)
            r.barrier()
            r.read(nx, t + 1)
        r.lgkm_wait()
        cur, t = nx, t + 1
    return r


@pytest.mark.parametrize("ns", [3, 4, 5, 6])
@pytest.mark.parametrize("nk", [1, 2, 3, 4, 5, 6, 7, 16, 64])
def test_gemm_mid_interleaved_ring_schedule(ns, nk):
    """The interleaved ring's slot / wait / barrier order (csrc/gemm_mid.hip ILV) keeps both ring invariants for
    every depth and k-step count, including split-K slices shorter than the ring."""
    r = _ilv_schedule(ns, 5, 5 + nk)
    assert sorted(r.issued) == list(range(5, 5 + nk))


def test_ring_model_catches_an_early_restage():
    """The model is not vacuous: restaging stage t-1's slot before the mid-k-step barrier is caught."""
    r = _RingModel(3)
    r.issue(0, 0), r.issue(1, 1)
    r.vm_wait(1), r.barrier(), r.read(0, 0)
    with pytest.raises(AssertionError):
        r.issue(2, 0)
