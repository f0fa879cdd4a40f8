"""Host-side plan logic (no GPU): autotuner candidate lists for the decode GEMM tiles and the workspace slots
that keep concurrently running kernel chains apart (ops/autotune.py, ops/hip.py)."""
import pytest

from llmss_amd.ops import autotune as A


def _tiles(cands):
    return {(nt >> 8) & 15 for nt, _ in cands if nt >> 8}


@pytest.mark.parametrize("M,N,K,glu", [(64, 12288, 4096, False), (64, 22016, 4096, True), (64, 4096, 11008, False),
                                       (512, 1536, 4096, False), (64, 6400, 1600, False)])
def test_candidates_cover_the_round3_tiles(M, N, K, glu):
    c = A.candidates(M, N, K, glu, False)
    assert len(set(c)) == len(c), "duplicate candidates"
    # the gemm_mid decode tiles: 64x192 (13), 64x32 (14), 64x96 (15), 64x48 (7), and the odd / large splits
    assert {7, 13, 14, 15} <= _tiles(c)
    nk = -(-K // 64)
    for nt, s in c:
        assert s >= 1 and (s == 1 or nk // s >= 1)
    if nk // 11 >= 2:
        assert any(s == 11 for _, s in c)


def test_qkv_epilogue_candidates_are_combined_or_unsplit():
    for nt, s in A.qkv_epi_candidates(64, 12288, 4096, 128, False):
        assert s == 1 or (nt >> 8) & 256, (hex(nt), s)  # a split plan must combine in-launch
    # neox RoPE needs head-aligned tiles: no 64x48 / 64x96 / 64x192 plans for D = 128
    neox = _tiles(A.qkv_epi_candidates(64, 12288, 4096, 128, True))
    assert not ({7, 13, 14, 15} & neox)


def test_w8a8_candidates_include_the_fp8_gemm_mid_tiles():
    from llmss_amd.ops.hip import W8A8_FLAG

    c = [nt for nt, _ in A.candidates(64, 10240, 8192, False, True) if nt & W8A8_FLAG]
    tiles = {(nt >> 8) & 15 for nt in c}
    assert {7, 10, 11, 13, 15} <= tiles
    assert not [nt for nt, _ in A.candidates(64, 10240, 8200, False, True) if nt & W8A8_FLAG and (nt >> 8) & 15 >= 7]


def test_workspace_slots_are_disjoint():
    from llmss_amd.ops import hip as H

    a0 = H._GEMM_WS._items[0]
    with H.workspace_slot(1):
        assert H._GEMM_WS._items[H._SLOT.k] is not a0
        with H.workspace_slot(2):
            assert H._SLOT.k == 2
        assert H._SLOT.k == 1
    assert getattr(H._SLOT, "k", 0) == 0


def test_interleaved_ring_candidates_only_where_the_kernel_takes_them():
    """Hint bit 512 (gemm_mid ILV) appears for M >= ILV_MIN_M, K % 64 == 0 and ring depths >= 3 only."""
    ilv = lambda c: [(n, s) for n, s in c if n & (512 << 8)]
    assert ilv(A.candidates(512, 1536, 4096, False, False))
    assert all(((n >> 8) & 48) >= 16 for n, _ in ilv(A.candidates(512, 1536, 4096, False, False)))
    assert not ilv(A.candidates(64, 1536, 4096, False, False))
    assert not ilv(A.candidates(512, 4096, 1376, False, False))  # partial last k-step


def test_prompt_batch_library_decision(monkeypatch):
    """ops/autotune.py tune_prefill_library: only plain projections are timed (no SwiGLU / activation / head),
    the library takes a shape when it is 3 % faster, and the caller's `agree` (a min over TP ranks) overrules a
    local win."""
    import types

    import torch

    from llmss_amd.ops import hip as H

    times = {(12288, 4096): (790.0, 580.0), (4096, 4096): (230.0, 229.0), (4096, 11008): (610.0, 480.0)}
    cur = {}

    def fake_time(fn, iters):
        fn(0)
        return cur.pop("t")

    def fake_linear(x, w, *a, **k):
        cur["t"] = times[tuple(w.shape)][0]

    def fake_matmul(x, wt, out=None):
        cur["t"] = times[tuple(wt.t().shape)][1]

    monkeypatch.setattr(A, "_time", fake_time)
    monkeypatch.setattr(H, "linear", fake_linear)
    monkeypatch.setattr(torch, "matmul", fake_matmul)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    A._DONE_LIB.clear()
    lin = lambda n, k, glu=False: types.SimpleNamespace(N=n, K=k, glu=glu, w_scale=None, packed=False)
    L = types.SimpleNamespace(qkv=lin(12288, 4096), o=lin(4096, 4096), up=lin(22016, 4096, True),
                              down=lin(4096, 11008))
    model = types.SimpleNamespace(device=torch.device("cpu"), tp=types.SimpleNamespace(size=1), act="silu",
                                  cfg=types.SimpleNamespace(parallel_block=False),
                                  w=types.SimpleNamespace(layers=[L], head=lin(32000, 4096)))
    H._LIB_PREFILL.clear()
    try:
        res = A.tune_prefill_library(model, 4096, iters=1)
        assert set(res) == {"qkv", "o", "down"}  # up (SwiGLU) and the head are not candidates
        assert H._LIB_PREFILL == {(12288, 4096), (4096, 11008)}  # o: within 3 %
        A.tune_prefill_library(model, 4096, agree=lambda f: 0, iters=1)  # a peer rank disagrees
        assert H._LIB_PREFILL == set()
        assert A.tune_prefill_library(model, 512) == {}  # decode-sized M: never
    finally:
        H._LIB_PREFILL.clear()
        A._DONE_LIB.clear()
