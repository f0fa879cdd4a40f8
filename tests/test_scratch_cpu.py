"""Scratch buffers that decode graphs capture (ops/hip.py) are grown by later eager calls - a prefill of 8192 rows
after the graphs of <= 64-row buckets were captured. The outgrown buffer must stay allocated: each captured graph
keeps writing to its old address on every replay, and a freed block would be handed to live tensors by the caching
allocator. Exercised with CPU tensors (the classes take the device)."""
import pytest

from llmss_amd.ops import hip as H


@pytest.mark.parametrize("make,grow", [
    (H._QuantScratch, lambda w, M: w.get(M, 64, "cpu")),
    (H._PreQScratch, lambda w, M: w.get(M, 64, "cpu")),
    (H._MxScratch, lambda w, M: w.get(M, 64, "cpu")),
    (H.DecodeWorkspace, lambda w, M: w.get(M, 4, 2, 64, "cpu")),
    (H.GemmWorkspace, lambda w, M: w.get(M << 20, "cpu")),
])
def test_outgrown_scratch_is_retired_not_freed(make, grow, monkeypatch):
    monkeypatch.setattr(H.torch.cuda, "is_current_stream_capturing", lambda: False)  # no device here
    w = make()
    small = grow(w, 4)
    small = small if isinstance(small, tuple) else (small,)
    ptrs = [t.untyped_storage().data_ptr() for t in small]
    big = grow(w, 64)
    big = big if isinstance(big, tuple) else (big,)
    assert big[0].untyped_storage().data_ptr() != ptrs[0]  # it did grow
    kept = {t.untyped_storage().data_ptr() for t in H._RETIRED}
    assert all(p in kept for p in ptrs)


def test_scratch_grows_geometrically(monkeypatch):
    """Prompt batches of every size from 1 to 1000 rows retire at most ~log2(1000) buffers, not one per size."""
    monkeypatch.setattr(H.torch.cuda, "is_current_stream_capturing", lambda: False)
    w = H._QuantScratch()
    n0 = len(H._RETIRED)
    for M in range(1, 1001):
        q, s = w.get(M, 64, "cpu")
        assert q.shape == (M, 64) and s.shape == (M,)
    assert len(H._RETIRED) - n0 <= 2 * 11
