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
    os.environ.update(env or {})  # e.g. the overlap paths
    torch.set_num_threads(1)
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model
    from llmss_amd.parallel.dist import initialize_distributed

    tp, r, w = initialize_distributed(backend="gloo")
    m = build_model(ckpt, tp, "fp32", "cpu")
    if "LLMSS_TP_DECODE_OVERLAP_MIN" in (env or {}):
        assert m.overlap_split(3) == 1  # the 3-sequence decode steps really take the micro-batch path
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64, check_tokens=True)
    greedy = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    sampled = eng.generate(prompts, [SamplingParams(max_new_tokens=8, temperature=0.9, top_k=20, top_p=0.9, seed=5 + i,
                                                    ignore_eos=True) for i in range(len(prompts))])
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


# LLMSS_TP_OVERLAP_ROWS: row-chunked prefill all-reduce / GEMM overlap;
# LLMSS_TP_DECODE_OVERLAP_MIN: decode steps as two interleaved micro-batches (the 3-sequence batch splits 1 + 2)
_ROWS = {"LLMSS_TP_OVERLAP_ROWS": "4"}
_TBO = {"LLMSS_TP_DECODE_OVERLAP_MIN": "2"}


@pytest.mark.parametrize("name,world,overlap", [("llama", 2, None), ("gptj", 2, None), ("bigcode", 4, None),
                                                ("gpt2", 2, None), ("bigcode_mha", 2, None), ("llama", 2, _ROWS),
                                                ("gptj", 2, {"LLMSS_TP_OVERLAP_ROWS": "5"}), ("llama", 2, _TBO),
                                                ("gptj", 2, _TBO), ("bigcode", 4, _TBO)])
def test_tp_matches_single(tmp_path, name, world, overlap):
    d = str(tmp_path / name)
    save_hf_model(name, d, vocab=101)  # 101 % world != 0 -> exercises the padded vocab-parallel head
    prompts = [[(3 * i + 7 * j) % 100 for j in range(5 + 2 * i)] for i in range(3)]
    from llmss_amd.engine import LLMEngine, SamplingParams, build_model

    m = build_model(d, None, "fp32", "cpu")
    eng = LLMEngine(m, max_num_seqs=4, block_size=4, num_blocks=64)
    ref_g = eng.generate(prompts, SamplingParams(max_new_tokens=8, is_greedy=True, ignore_eos=True))
    ref_s = eng.generate(prompts, [SamplingParams(max_new_tokens=8, temperature=0.9, top_k=20, top_p=0.9, seed=5 + i,
                                                  ignore_eos=True) for i in range(len(prompts))])
    g, s = _run(world, d, prompts, overlap)
    assert g == ref_g
    assert s == ref_s
