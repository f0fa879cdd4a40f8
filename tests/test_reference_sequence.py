"""The reference's own call sequence against the import-compatible façade (``llmss.server.models.utils.dist``):
``generate.py:42-67`` - ``initialize_torch_distributed()`` -> ``torch.distributed.barrier(process_group)`` ->
``weight_files`` -> ``Weights(..., process_group)`` -> ``MODEL_REGISTRY[type](config, weights)`` -> ``eval()`` ->
(world > 1) ``dist.broadcast(input_ids, src=0)`` -> forward - at world size 1 (FakeGroup, no default process
group, like the reference) and world size 2 (gloo, the world ProcessGroup handed out), plus the reference
``FakeGroup`` API itself (``dist.py:14-37``)."""
import os
import socket

import torch
import torch.multiprocessing as mp
from transformers import AutoConfig

from helpers import save_hf_model


def test_fake_group_reference_api():
    from llmss.server.models.utils.dist import FakeBarrier, FakeGroup, as_tp_group

    g = FakeGroup(1, 2)
    assert g.size() == 2 and g.rank() == 1
    assert isinstance(g.allreduce(torch.ones(3)), FakeBarrier)
    g.barrier().wait()
    out = [[torch.zeros(2)]]
    g.allgather(out, [torch.tensor([3.0, 4.0])]).wait()
    assert out[0][0].tolist() == [3.0, 4.0]
    tp = as_tp_group(g)
    assert (tp.rank, tp.size, tp.fake) == (1, 2, True)
    tp1 = as_tp_group(FakeGroup(0, 1))
    assert (tp1.size, tp1.is_real) == (1, False)


def _sequence(d, prompt, tp_size=None):
    """generate.py:42-67 + one cached forward; returns (world_size, rank, logits). ``tp_size``: the expected
    tensor-parallel width of the returned process group (world size unless data-parallel replicas are on)."""
    from llmss.server.models.custom_modeling import MODEL_REGISTRY
    from llmss.server.models.utils.dist import initialize_torch_distributed
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    process_group, rank, world_size = initialize_torch_distributed()
    torch.distributed.barrier(process_group)  # generate.py:62 (a FakeGroup at world 1, as in the reference)
    device, dtype = torch.device("cpu"), torch.float32
    config = AutoConfig.from_pretrained(d)
    weights = Weights(weight_files(d), device=device, dtype=dtype, process_group=process_group)
    tp_size = tp_size or world_size
    assert weights.process_group.size() == tp_size and weights.process_group.rank() == rank % tp_size
    model = MODEL_REGISTRY[config.model_type](config, weights)
    model.eval()
    ids = prompt.clone() if rank == 0 else torch.zeros_like(prompt)
    if world_size > 1:
        torch.distributed.broadcast(ids, src=0)  # generate.py:85 (needs the default group: world > 1 only)
    out = model(ids, use_cache=True)
    nxt = out.logits[:, -1:].argmax(-1)
    out2 = model(nxt, past_key_values=out.past_key_values, use_cache=True)
    return world_size, rank, torch.cat([out.logits, out2.logits], 1)


def _worker(rank, port, d, prompt, q, world=2, dp=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LLMSS_DP=str(dp))
    torch.set_num_threads(1)
    try:
        ws, r, logits = _sequence(d, prompt, world // dp)
        q.put((r, ws, logits.numpy()))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, -1, repr(e)))


def test_reference_generate_sequence_world1_and_world2(tmp_path, monkeypatch):
    d = str(tmp_path / "llama")
    hf = save_hf_model("llama", d, vocab=101)  # 101 % 2 != 0: padded vocab-parallel head at world 2
    prompt = torch.randint(0, 100, (2, 7))
    with torch.no_grad():
        full = hf(prompt).logits
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ws, r, ref = _sequence(d, prompt)
    assert (ws, r) == (1, 0)
    assert not torch.distributed.is_initialized()  # world 1: FakeGroup, no default group (reference dist.py:59-60)
    torch.testing.assert_close(ref[:, :7], full, rtol=1e-4, atol=1e-4)

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(i, port, d, prompt, q)) for i in range(2)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=240) for _ in range(2)]
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    for rank, ws2, logits in got:
        assert ws2 == 2, logits
        torch.testing.assert_close(torch.from_numpy(logits), ref, rtol=1e-4, atol=1e-4)  # TP=2 over gloo == world 1
    assert [p.exitcode for p in procs] == [0, 0]


def test_reference_generate_sequence_dp2(tmp_path):
    """World 4 with two data-parallel replicas (LLMSS_DP=2): initialize_torch_distributed hands each rank its
    replica's group (TP=2), not the world, so Weights / MODEL_REGISTRY shard over 2 ranks and every replica
    computes the world-1 logits."""
    d = str(tmp_path / "llama")
    save_hf_model("llama", d, vocab=101)
    prompt = torch.randint(0, 100, (2, 7))
    with torch.no_grad():
        from transformers import AutoModelForCausalLM

        full = AutoModelForCausalLM.from_pretrained(d, torch_dtype=torch.float32)(prompt).logits
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(i, port, d, prompt, q, 4, 2)) for i in range(4)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=300) for _ in range(4)]
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    for rank, ws, logits in got:
        assert ws == 4, logits
        torch.testing.assert_close(torch.from_numpy(logits)[:, :7], full, rtol=1e-4, atol=1e-4)
    assert [p.exitcode for p in procs] == [0] * 4
