"""Reference API surface beyond MODEL_REGISTRY: multi-token continuation of a cached prefix in ONE
call (paged extend step), ``attention_mask`` / ``position_ids`` honoured, the ``Weights`` shard
accessors and the tensor-parallel layer library (``llmss.server.models.utils.layers``) - on CPU
against HF / plain torch, and at TP=2 over gloo against TP=1."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
from transformers import AutoConfig

from helpers import save_hf_model


def _load(d, pg=None):
    from llmss.server.models.custom_modeling import MODEL_REGISTRY
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    config = AutoConfig.from_pretrained(d)
    w = Weights(weight_files(d), torch.device("cpu"), torch.float32, pg)
    return MODEL_REGISTRY[config.model_type](config, w), w


@pytest.mark.parametrize("name", ["llama", "gptj", "bigcode"])
def test_multi_token_continuation_one_call(tmp_path, name):
    d = str(tmp_path / name)
    hf = save_hf_model(name, d)
    model, _ = _load(d)
    ids = torch.randint(0, 100, (2, 13))
    out = model(ids[:, :6], use_cache=True)
    out2 = model(ids[:, 6:], past_key_values=out.past_key_values, use_cache=True)  # 7 tokens over a cached prefix
    with torch.no_grad():
        ref = hf(ids).logits
    torch.testing.assert_close(out2.logits, ref[:, 6:], rtol=1e-4, atol=1e-4)
    # rows at different depths in one call: row 0 decodes one token, row 1 continues with 3
    model.release(out2.past_key_values)


@pytest.mark.parametrize("name", ["bigcode", "llama"])
def test_attention_mask_left_padding(tmp_path, name):
    d = str(tmp_path / name)
    hf = save_hf_model(name, d)
    model, _ = _load(d)
    a = torch.randint(0, 100, (9,))
    b = torch.randint(0, 100, (5,))
    ids = torch.zeros(2, 9, dtype=torch.long)
    ids[0] = a
    ids[1, 4:] = b  # left padded
    mask = torch.ones(2, 9, dtype=torch.long)
    mask[1, :4] = 0
    out = model(ids, attention_mask=mask)
    with torch.no_grad():
        ra, rb = hf(a[None]).logits[0], hf(b[None]).logits[0]
    torch.testing.assert_close(out.logits[0], ra, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out.logits[1, 4:], rb, rtol=1e-4, atol=1e-4)
    assert out.logits[1, :4].abs().max() == 0  # padded positions are not computed


def test_position_ids_override(tmp_path):
    d = str(tmp_path / "gpt2")
    hf = save_hf_model("gpt2", d)
    model, _ = _load(d)
    ids = torch.randint(0, 100, (1, 6))
    pos = torch.arange(3, 9)[None]
    out = model(ids, position_ids=pos)
    with torch.no_grad():
        ref = hf(ids, position_ids=pos).logits
    torch.testing.assert_close(out.logits, ref, rtol=1e-4, atol=1e-4)


def test_weights_shard_accessors(tmp_path):
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    d = str(tmp_path / "gptj")
    save_hf_model("gptj", d)
    from llmss_amd.parallel.dist import TPGroup

    full = Weights(weight_files(d), torch.device("cpu"), torch.float32, None)
    name = "transformer.h.0.attn.q_proj.weight"
    W = full.get_tensor(name)
    for r in range(2):
        w = Weights(weight_files(d), torch.device("cpu"), torch.float32, TPGroup(r, 2, fake=True))
        assert w.process_group.size() == 2 and w.process_group.rank() == r
        torch.testing.assert_close(w.get_sharded(name, dim=0), W.chunk(2, 0)[r])
        torch.testing.assert_close(w.get_sharded(name, dim=1), W.chunk(2, 1)[r])
        torch.testing.assert_close(w.get_multi_weights_row("transformer.h.0.attn.out_proj"),
                                   full.get_tensor("transformer.h.0.attn.out_proj.weight").chunk(2, 1)[r])
        qkv = w.get_multi_weights_col([f"transformer.h.0.attn.{p}_proj" for p in "qkv"], dim=0)
        assert qkv.shape == (3 * W.shape[0] // 2, W.shape[1])
        assert w.get_filename(name)[1] == name and w.get_shape(name) == list(W.shape)
    w3 = Weights(weight_files(d), torch.device("cpu"), torch.float32, TPGroup(0, 3, fake=True))
    with pytest.raises(AssertionError):
        w3.get_sharded(name, dim=0)  # 64 rows over 3 ranks
    with pytest.raises(NotImplementedError):
        w3.get_partial_sharded("transformer.wte.weight", dim=2)


def _layers_forward(w, cfg_dir, x, ids):
    from llmss.server.models.utils.layers import (TensorParallelColumnLinear, TensorParallelEmbedding,
                                                  TensorParallelHead, TensorParallelRowLinear)

    emb = TensorParallelEmbedding("transformer.wte", w)
    fc_in = TensorParallelColumnLinear.load(None, "transformer.h.0.mlp.fc_in", w, bias=True)
    fc_out = TensorParallelRowLinear.load(None, "transformer.h.0.mlp.fc_out", w, bias=True)
    qkv = TensorParallelColumnLinear.load_multi(None, [f"transformer.h.0.attn.{p}_proj" for p in "qkv"], w,
                                                bias=False, dim=0)
    head = TensorParallelHead.load(None, "lm_head", w)
    ln = torch.nn.LayerNorm.load(prefix="transformer.h.0.ln_1", weights=w, eps=1e-5)
    h, res = ln(x)
    return emb(ids), fc_out(torch.nn.functional.gelu(fc_in(h))), qkv(h).shape, head(h), res


def _layers_worker(rank, port, d, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    torch.set_num_threads(1)
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights
    from llmss_amd.parallel.dist import initialize_distributed

    tp, _, _ = initialize_distributed(backend="gloo")
    w = Weights(weight_files(d), torch.device("cpu"), torch.float32, tp)
    torch.manual_seed(0)
    x = torch.randn(3, 64)
    ids = torch.tensor([[1, 50, 100]])
    out = _layers_forward(w, d, x, ids)
    if rank == 0:
        q.put(out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_tp_layer_library_tp2_matches_tp1(tmp_path):
    from llmss.server.models.utils.hub import weight_files
    from llmss.server.models.utils.weights import Weights

    d = str(tmp_path / "gptj")
    save_hf_model("gptj", d, vocab=101)  # 101 % 2 != 0: padded vocab-parallel head
    w = Weights(weight_files(d), torch.device("cpu"), torch.float32, None)
    torch.manual_seed(0)
    x = torch.randn(3, 64)
    ids = torch.tensor([[1, 50, 100]])
    ref = _layers_forward(w, d, x, ids)
    # TP=1 layers == plain torch
    W = w.get_tensor("lm_head.weight")
    ln = torch.nn.functional.layer_norm(x, (64,), w.get_tensor("transformer.h.0.ln_1.weight"),
                                        w.get_tensor("transformer.h.0.ln_1.bias"), 1e-5)
    torch.testing.assert_close(ref[3], ln @ W.t())
    torch.testing.assert_close(ref[4], x)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_layers_worker, args=(r, port, d, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=240)
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    assert [p.exitcode for p in procs] == [0, 0]
    torch.testing.assert_close(got[0], ref[0])  # embedding (replicated table, no all-reduce)
    torch.testing.assert_close(got[1], ref[1], rtol=1e-5, atol=1e-5)  # column -> row + all-reduce (+ rank-0 bias)
    assert got[2][1] * 2 == ref[2][1]  # fused q|k|v column shard
    torch.testing.assert_close(got[3], ref[3], rtol=1e-5, atol=1e-5)  # vocab-parallel head, padded then trimmed


def test_pool_exhaustion_leaves_pool_intact(tmp_path):
    """a call that cannot get its KV blocks raises without leaking the blocks of earlier rows."""
    d = str(tmp_path / "llama")
    save_hf_model("llama", d)
    model, _ = _load(d)
    free0 = len(model._free)
    ids = torch.randint(0, 100, (3, (free0 // 3 + 2) * model.block_size))  # needs more blocks than the pool has
    with pytest.raises(RuntimeError, match="exhausted"):
        model(ids, use_cache=True)
    assert len(model._free) == free0
    out = model(ids[:, :20], use_cache=True)  # the pool still serves a call that fits
    model.release(out.past_key_values)
    assert len(model._free) == free0
