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


def test_w8a8_software_pipelined_candidates_are_4_wave_gemm_mid_tiles():
    """W8A8_ILV (the fp8 gemm_mid k-loop with the next step's reads between the MFMAs) is a candidate for M >= 128
    on the 4-wave gemm_mid tiles only: the 8-wave ones spill its second fragment set (profiles/r6_f8)."""
    from llmss_amd.ops.hip import W8A8_FLAG, W8A8_ILV

    c = [(n, s) for n, s in A.candidates(512, 7168, 8192, True, True) if n & W8A8_FLAG and n & W8A8_ILV]
    tiles = {(n >> 8) & 15 for n, _ in c}
    assert 8 in tiles and 11 in tiles and not tiles & {9, 12} and tiles <= {7, 8, 10, 11, 13, 15}
    assert all(3 <= (n >> 12) & 15 <= 5 for n, _ in c)
    assert not [n for n, _ in A.candidates(64, 7168, 8192, True, True) if n & W8A8_FLAG and n & W8A8_ILV]


@pytest.mark.parametrize("col", ["4", "0"])
def test_model_shapes_include_the_column_chunks_when_forced(monkeypatch, col):
    """The autotuner tunes o / down's column slices (DecoderLM._reduce_cols) whenever the column schedule can run."""
    import torch

    from llmss_amd.models.config import get_preset
    from llmss_amd.models.decoder import DecoderLM
    from llmss_amd.models.weights import random_weights
    from llmss_amd.parallel.dist import TPGroup

    monkeypatch.setenv("LLMSS_TP_COL", col)
    cfg = get_preset("llama2-7b", num_layers=1, hidden_size=256, intermediate_size=512, num_heads=4, head_dim=64,
                     num_kv_heads=4, rotary_dim=64, vocab_size=512, max_position_embeddings=64)
    tp = TPGroup(0, 2, fake=True, sim_comm=(15.0, 150.0))
    m = DecoderLM(cfg, random_weights(cfg, tp=2, rank=0, dtype=torch.float32, seed=0), tp)
    shapes = A.model_shapes(m)
    L = m.w.layers[0]
    if col == "0":
        assert "o_col" not in shapes and "down_col" not in shapes
    else:
        assert shapes["o_col"] == A.GemmShape(L.o.N // 4, L.o.K)
        assert shapes["down_col"] == A.GemmShape(L.down.N // 4, L.down.K)


@pytest.mark.parametrize("M,N,K", [(65536, 4096, 1376), (8192, 4096, 4096), (65536, 1536, 4096), (8192, 1600, 1600)])
def test_prompt_batch_plans_take_the_ping_pong_kernel(M, N, K):
    """Every prompt-batch projection with enough 256x256 tiles runs the ping-pong kernel (tile code 4), including
    K % 64 != 0 (Llama-2-7B's TP=8 down projection, K = 1376: its partial last K-tile reads a zero page; before
    round 5 it fell back to the 128x128 kernel, profiles/r5_prefill_tp8)."""
    from llmss_amd.ops import hip as H

    nt, split = H.lib().gemm_plan(M, N, K, False)
    assert (nt >> 8) & 15 == 4 and split == 1, (hex(nt), split)
