"""Native C++ runtime: block allocator, continuous-batching scheduler, safetensors reader."""
import numpy as np
import pytest
import torch


def test_block_allocator(native):
    a = native.BlockAllocator(8, 16)
    bs = a.allocate_n(5)
    assert len(set(bs)) == 5 and a.num_free() == 3
    a.fork(bs[0])
    a.free(bs[0])
    assert a.ref_count(bs[0]) == 1 and a.num_free() == 3
    a.free_all(bs)
    assert a.num_free() == 8
    with pytest.raises(RuntimeError):
        a.free(bs[1])
    with pytest.raises(RuntimeError):
        a.allocate_n(9)


def test_scheduler_prefill_then_decode(native):
    s = native.Scheduler(num_blocks=64, block_size=4, max_num_seqs=8, max_batched_tokens=64, max_model_len=64)
    s.add(10, 5, 3)
    s.add(11, 9, 3)
    b = s.schedule()
    assert b.kind == 1 and b.ids.tolist() == [10, 11] and b.query_lens.tolist() == [5, 9]
    assert b.positions.tolist() == list(range(5)) + list(range(9))
    bt = b.block_table
    slots = b.slots.tolist()
    # slots follow the block table
    assert slots[:5] == [bt[0, p // 4] * 4 + p % 4 for p in range(5)]
    s.on_token(10, False)
    s.on_token(11, False)
    b = s.schedule()
    assert b.kind == 2 and b.ctx_lens.tolist() == [6, 10] and b.positions.tolist() == [5, 9]
    s.on_token(10, True)  # finished early (eos)
    s.on_token(11, False)
    b = s.schedule()
    assert b.ids.tolist() == [11]
    s.on_token(11, False)  # third token -> length limit
    assert not s.has_work()
    assert s.num_free_blocks() == 64


def test_scheduler_budget_and_preemption(native):
    s = native.Scheduler(num_blocks=6, block_size=4, max_num_seqs=4, max_batched_tokens=16, max_model_len=32)
    s.add(1, 8, 16)
    s.add(2, 8, 16)
    s.add(3, 8, 16)
    b = s.schedule()
    assert b.kind == 1 and b.ids.tolist() == [1, 2]  # token budget 16
    assert b.sample.tolist() == [True, True] and b.num_decode == 0
    for i in b.ids.tolist():
        s.on_token(i, False)
    b = s.schedule()  # decodes first: 1 and 2 take the last 2 blocks, 3 cannot be admitted
    assert b.kind == 2 and b.ids.tolist() == [1, 2] and s.num_waiting() == 1
    preempted = []
    for _ in range(8):
        for i in b.ids.tolist():
            s.on_token(i, False)
        b = s.schedule()
        preempted += b.preempted.tolist()
        if preempted:
            break
    assert preempted == [2]  # the newest running sequence is recomputed later
    assert b.ids.tolist() == [1]
    assert s.num_waiting() == 2


def test_scheduler_chunked_prefill_and_mixed_steps(native):
    s = native.Scheduler(num_blocks=64, block_size=4, max_num_seqs=4, max_batched_tokens=10, max_model_len=64)
    s.add(1, 25, 4)
    chunks = []
    while True:
        b = s.schedule()
        assert b.kind == 1 and b.ids.tolist() == [1]
        chunks.append((b.query_lens.tolist(), b.positions.tolist()[0], b.ctx_lens.tolist(), b.sample.tolist()))
        if b.sample[0]:
            break
        assert s.num_prefilling() == 1
    assert chunks == [([10], 0, [10], [False]), ([10], 10, [20], [False]), ([5], 20, [25], [True])]
    s.on_token(1, False)
    assert s.num_prefilling() == 0
    s.add(2, 12, 4)
    b = s.schedule()  # the decode of 1 rides along with the first chunk of 2
    assert b.kind == 1 and b.num_decode == 1 and b.ids.tolist() == [1, 2]
    assert b.query_lens.tolist() == [1, 9] and b.sample.tolist() == [True, False]
    assert b.positions.tolist()[:2] == [25, 0] and b.ctx_lens.tolist() == [26, 9]
    s.on_token(1, False)
    b = s.schedule()
    assert b.ids.tolist() == [1, 2] and b.query_lens.tolist() == [1, 3] and b.sample.tolist() == [True, True]
    # slots of a chunk continue the sequence's blocks
    bt = b.block_table[1]
    assert b.slots.tolist()[1:] == [int(bt[p // 4]) * 4 + p % 4 for p in range(9, 12)]


def test_scheduler_whole_prompt_mode(native):
    s = native.Scheduler(64, 4, 4, 10, 64, -1)
    with pytest.raises(ValueError):
        s.add(1, 25, 4)  # longer than the per-step budget
    s.add(2, 8, 4)
    s.add(3, 8, 4)
    b = s.schedule()
    assert b.ids.tolist() == [2] and b.query_lens.tolist() == [8]  # 3 does not fit whole


def test_scheduler_rejects_too_long(native):
    s = native.Scheduler(16, 4, 4, 64, 16)
    with pytest.raises(ValueError):
        s.add(1, 10, 10)


def test_safetensors_reader(native, tmp_path):
    from safetensors.torch import save_file

    t = {"a": torch.randn(7, 5), "b.c": torch.arange(24, dtype=torch.int64).view(2, 3, 4),
         "h": torch.randn(6, 9).to(torch.bfloat16)}
    p = str(tmp_path / "x.safetensors")
    save_file(t, p, metadata={"format": "pt"})
    f = native.SafetensorsFile(p)
    assert sorted(f.keys()) == ["a", "b.c", "h"]
    assert f.metadata()["format"] == "pt"
    from llmss_amd.utils.checkpoint import CheckpointReader

    r = CheckpointReader([p])
    assert torch.equal(r.get("a"), t["a"])
    assert torch.equal(r.rows("a", 2, 5), t["a"][2:5])
    assert torch.equal(r.cols("a", 1, 4), t["a"][:, 1:4])
    assert torch.equal(r.cols("b.c", 1, 3), t["b.c"][:, 1:3])
    assert torch.equal(r.cols("h", 3, 9), t["h"][:, 3:9])
    assert r.shape("b.c") == [2, 3, 4]


def test_step_seeds_vectorised_matches_scalar():
    import random

    import numpy as np

    from llmss_amd.engine.sampling import step_seed, step_seeds

    rng = random.Random(3)
    seeds = [rng.getrandbits(64) for _ in range(500)] + [0, (1 << 64) - 1]
    steps = [rng.randint(0, 10_000) for _ in range(500)] + [0, 7]
    got = step_seeds(np.array(seeds, dtype=np.uint64), np.array(steps, dtype=np.int64)).tolist()
    assert got == [step_seed(s, t) for s, t in zip(seeds, steps)]


def test_scheduler_on_tokens_batched():
    import numpy as np

    from llmss_amd import _native

    S = _native().Scheduler(64, 4, 8, 64, 32)
    for i in range(3):
        S.add(i, 5, 3)
    b = S.schedule()
    assert b.kind == 1
    S.on_tokens(b.ids, np.array([False, True, False]))  # request 1 stops early (eos)
    b = S.schedule()
    assert b.kind == 2 and b.ids.tolist() == [0, 2]
    S.on_tokens(b.ids, np.zeros(2, dtype=bool))
    b = S.schedule()
    S.on_tokens(b.ids, np.zeros(2, dtype=bool))  # third token: max_new reached -> finished
    assert not S.has_work()


def _drive(s, max_steps=500):
    """Run the scheduler to completion as the engine would; every step must do work."""
    steps = preempted = 0
    while s.has_work():
        b = s.schedule()
        assert b.kind != 0, "idle step with work left (livelock)"
        preempted += len(b.preempted)
        for i, smp in zip(b.ids.tolist(), b.sample.tolist()):
            if smp:
                s.on_token(i, False)
        steps += 1
        assert steps < max_steps
    return steps, preempted


@pytest.mark.parametrize("chunk", [8, 0])
def test_scheduler_chunked_prefill_pool_exhaustion(native, chunk):
    """concurrent chunked prompts that together hold the whole KV pool while nothing
    decodes used to make every later schedule() idle forever. Now the newest is preempted."""
    s = native.Scheduler(num_blocks=8, block_size=4, max_num_seqs=4, max_batched_tokens=16, max_model_len=64,
                         prefill_chunk=chunk)
    s.add(1, 20, 4)
    s.add(2, 20, 4)
    steps, preempted = _drive(s)
    assert preempted >= 1 and s.num_free_blocks() == 8


def test_scheduler_rejects_sequence_larger_than_pool(native):
    s = native.Scheduler(num_blocks=4, block_size=4, max_num_seqs=4, max_batched_tokens=64, max_model_len=64)
    with pytest.raises(ValueError):
        s.add(1, 16, 4)  # 20 tokens need 5 blocks; the pool has 4
    s.add(2, 12, 4)
    assert _drive(s)[0] > 0


def test_scheduler_reserve_ahead_of_schedule(native):
    """Scheduler.reserve: the pipelined decode takes the next KV block of a sequence before schedule() runs; the
    scheduler's next decode step uses that same block (no second allocation), an empty pool refuses (-1), and the
    reserved block is returned with the sequence."""
    s = native.Scheduler(num_blocks=3, block_size=4, max_num_seqs=2, max_batched_tokens=16, max_model_len=16)
    s.add(1, 4, 8)  # a full first block
    b = s.schedule()
    assert b.kind == 1 and s.num_free_blocks() == 2
    s.on_token(1, False)
    blk = s.reserve(1, 5)  # token 4 opens block 1
    assert blk >= 0 and s.num_free_blocks() == 1 and s.blocks(1)[1] == blk
    assert s.reserve(1, 5) == blk and s.num_free_blocks() == 1  # idempotent
    b = s.schedule()
    assert b.kind == 2 and b.slots.tolist() == [blk * 4] and s.num_free_blocks() == 1
    assert s.reserve(1, 9) >= 0 and s.num_free_blocks() == 0
    assert s.reserve(1, 13) == -1  # pool empty: no preemption here
    assert s.reserve(1, 17) == -1  # past max_model_len
    s.finish(1)
    assert s.num_free_blocks() == 3
