"""Tensor parallelism over real multi-process collectives (gloo on CPU): TP=2/4 logits and greedy
continuations must equal TP=1 for every family (column/row/vocab-parallel sharding, GQA/MQA
head placement, single all-reduce for the GPT-J parallel block, padded vocab-parallel head)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from helpers import FAMILIES, save_hf_model


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ckpt, prompts, q, env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    env = dict(env or {})
    attrs = {k: int(env.pop(k)) for k in ("overlap_rows", "tbo_min") if k in env}  # DecoderLM attributes
    os.environ.update(env)  # e.g. the overlap paths
    torch.set_num_threads(1)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed

    tp, r, w = initialize_distributed(backend="gloo")
    m = build_model(ckpt, tp, "fp32", "cpu")
    for k, v in attrs.items():
        setattr(m, k, v)
    if "tbo_min" in attrs:
        assert m.overlap_split(3) == 1  # the 3-sequence decode steps really take the micro-batch path
    if "LLMSS_TP_PREFILL_OVERLAP_MIN" in (env or {}):  # the 3-prompt prefill splits at a sequence boundary
        from llmss_amd.models.decoder import StepInput
        assert m.prefill_split(StepInput("prefill", *(torch.zeros(21),) * 3, cu_host=[0, 5, 12, 21])) == (2, 12)
    calls = [0]
    if (env or {}).get("LLMSS_TP_RSAG") == "1":  # the row-sharded decode schedule really runs
        inner = m._hidden_states_rsag
        m._hidden_states_rsag = lambda *a_, **k_: (calls.__setitem__(0, calls[0] + 1), inner(*a_, **k_))[1]
    if (env or {}).get("LLMSS_TP_COL"):  # the column-chunked decode schedule really runs
        inner_c = m._reduce_cols
        m._reduce_cols = lambda *a_, **k_: (calls.__setitem__(0, calls[0] + 1), inner_c(*a_, **k_))[1]
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64, check_tokens=True)
    greedy = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    sampled = eng.generate(prompts, [SamplingParams(max_new_tokens=8, temperature=0.9, top_k=20, top_p=0.9, seed=5 + i,
                                                    ignore_eos=True) for i in range(len(prompts))])
    if (env or {}).get("LLMSS_TP_RSAG") == "1" or (env or {}).get("LLMSS_TP_COL"):
        assert calls[0] > 0, "the forced decode schedule never ran"
    # comm-stream fork / join structure (models/decoder.py StreamLedger): everything forked was joined, and the
    # schedules that overlap collectives really forked (the same calls fork and join streams on the GPU)
    assert not m._ledger.open
    if attrs or any(k in env for k in ("LLMSS_TP_BUCKET_BYTES", "LLMSS_TP_PREFILL_OVERLAP_MIN", "LLMSS_TP_COL")):
        assert m._ledger.forks > 0, "the overlapped schedule never forked the comm stream"
    if r == 0:
        q.put((greedy, sampled))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _run(world, ckpt, prompts, env=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ckpt, prompts, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


# overlap_rows (DecoderLM attribute) / LLMSS_TP_BUCKET_BYTES: row-bucketed all-reduce / GEMM overlap (rows, or bytes
# per bucket); tbo_min (attribute): decode steps as two interleaved micro-batches (the 3-sequence batch splits 1 + 2)
_ROWS = {"overlap_rows": "4"}
_TBO = {"tbo_min": "2"}
_PTBO = {"LLMSS_TP_PREFILL_OVERLAP_MIN": "2"}  # prefill steps as two micro-batches split at a sequence boundary
_RSAG = {"LLMSS_TP_RSAG": "1"}  # row-sharded decode: reduce-scatter -> add + norm on M / tp rows -> all-gather
_COL = {"LLMSS_TP_COL": "2"}  # column-chunked decode: row-parallel outputs as 2 weight-row slices, one AR each


@pytest.mark.parametrize("name,world,overlap", [("llama", 2, None), ("gptj", 2, None), ("bigcode", 4, None),
                                                ("gpt2", 2, None), ("bigcode_mha", 2, None), ("llama", 2, _ROWS),
                                                ("gptj", 2, {"overlap_rows": "5"}), ("llama", 2, _TBO),
                                                ("llama", 2, {"LLMSS_TP_BUCKET_BYTES": "64"}),
                                                ("gptj", 2, _TBO), ("bigcode", 4, _TBO), ("llama", 2, _PTBO),
                                                ("gptj", 2, _PTBO), ("bigcode", 4, {**_PTBO, **_TBO}),
                                                ("llama", 2, _RSAG), ("gptj", 2, _RSAG), ("bigcode", 4, _RSAG),
                                                ("gpt2", 4, _RSAG), ("llama", 2, _COL), ("gpt2", 2, _COL),
                                                ("bigcode", 4, {"LLMSS_TP_COL": "4"}),
                                                # the full node: TP=8 (one kv head per rank), plain and overlapped
                                                ("llama16", 8, None), ("llama16", 8, _TBO),
                                                ("llama16", 8, {"LLMSS_TP_COL": "2"})])
def test_tp_matches_single(tmp_path, name, world, overlap):
    d = str(tmp_path / name)
    save_hf_model(name, d, vocab=101)  # 101 % world != 0 -> exercises the padded vocab-parallel head
    # the row-sharded schedule needs decode batches divisible by the TP degree: 4 sequences
    n = 4 if overlap is not None and "LLMSS_TP_RSAG" in overlap else 3
    prompts = [[(3 * i + 7 * j) % 100 for j in range(5 + 2 * i)] for i in range(n)]
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    m = build_model(d, None, "fp32", "cpu")
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64)
    ref_g = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    ref_s = eng.generate(prompts, [SamplingParams(max_new_tokens=8, temperature=0.9, top_k=20, top_p=0.9, seed=5 + i,
                                                  ignore_eos=True) for i in range(len(prompts))])
    g, s = _run(world, d, prompts, overlap)
    assert g == ref_g
    assert s == ref_s


def _consistency_worker(rank, world, port, ckpt, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed

    tp, r, w = initialize_distributed(backend="gloo")
    m = build_model(ckpt, tp, "fp32", "cpu")
    try:
        if mode == "blocks":
            # each rank sizes its KV pool from its own (here: deliberately different) free memory;
            # 9 blocks of 4 tokens on rank 0 forces preemption for these 3 prompts x 13 tokens
            LLMEngine._auto_blocks = lambda self, frac: 9 if r == 0 else 200 + 50 * r
            eng = LLMEngine(m, max_num_seqs=4, block_size=4, check_tokens=True)
            prompts = [[(3 * i + 7 * j) % 100 for j in range(5 + 2 * i)] for i in range(3)]
            out = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
            q.put((r, eng.num_blocks, eng.stats["preemptions"], out))
        else:  # rank 1 runs a different engine config: must raise on every rank, not hang
            LLMEngine(m, max_num_seqs=4 if r == 0 else 8, block_size=4, num_blocks=64)
            q.put((r, "no error"))
    except RuntimeError as e:
        q.put((r, "raised", str(e)[:200]))
    torch.distributed.destroy_process_group()


def _run_consistency(world, ckpt, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_consistency_worker, args=(r, world, port, ckpt, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(10)
    return res, [p.exitcode for p in procs]


def test_kv_pool_agreed_across_ranks(tmp_path):
    d = str(tmp_path / "llama")
    save_hf_model("llama", d, vocab=101)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    prompts = [[(3 * i + 7 * j) % 100 for j in range(5 + 2 * i)] for i in range(3)]
    ref = LLMEngine(build_model(d, None, "fp32", "cpu"), max_num_seqs=4, block_size=4, num_blocks=64)
    ref_g = ref.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    res, codes = _run_consistency(2, d, "blocks")
    assert codes == [0, 0], res
    assert [x[1] for x in res] == [9, 9]  # the minimum of the ranks' own sizes
    assert res[0][2] > 0 and res[0][2] == res[1][2]  # same preemption decisions on both ranks
    assert res[0][3] == res[1][3] == ref_g


def test_mismatched_engine_config_raises(tmp_path):
    d = str(tmp_path / "gpt2")
    save_hf_model("gpt2", d, vocab=101)
    res, codes = _run_consistency(2, d, "mismatch")
    assert [x[1] for x in res] == ["raised", "raised"], res
    assert "max_num_seqs" in res[0][2]
