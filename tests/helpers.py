"""Test fixtures: tiny random HF checkpoints (+ an offline byte-level BPE tokenizer)."""
import os

import torch

FAMILIES = ["gpt2", "gptj", "bigcode", "bigcode_mha", "llama"]


def make_hf_model(name: str, vocab: int = 101, seed: int = 0):
    from transformers import (GPT2Config, GPT2LMHeadModel, GPTBigCodeConfig, GPTBigCodeForCausalLM, GPTJConfig,
                              GPTJForCausalLM, LlamaConfig, LlamaForCausalLM)

    torch.manual_seed(seed)
    if name == "gpt2":
        m = GPT2LMHeadModel(GPT2Config(n_embd=64, n_layer=2, n_head=4, n_positions=64, vocab_size=vocab,
                                       bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    elif name == "gptj":
        m = GPTJForCausalLM(GPTJConfig(n_embd=64, n_layer=2, n_head=4, n_positions=64, vocab_size=vocab, rotary_dim=8,
                                       bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    elif name == "bigcode":
        m = GPTBigCodeForCausalLM(GPTBigCodeConfig(n_embd=64, n_layer=2, n_head=4, n_positions=64, vocab_size=vocab,
                                                   multi_query=True, bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    elif name == "bigcode_mha":
        m = GPTBigCodeForCausalLM(GPTBigCodeConfig(n_embd=64, n_layer=2, n_head=4, n_positions=64, vocab_size=vocab,
                                                   multi_query=False, bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    elif name == "llama":
        m = LlamaForCausalLM(LlamaConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                         num_key_value_heads=2, intermediate_size=160, vocab_size=vocab,
                                         max_position_embeddings=64, bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    elif name == "llama16":  # TP up to 8: 16 q / 8 kv heads (2 q heads and 1 kv head per rank at TP=8)
        m = LlamaForCausalLM(LlamaConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=16,
                                         num_key_value_heads=8, intermediate_size=256, vocab_size=vocab,
                                         max_position_embeddings=64, bos_token_id=vocab - 1, eos_token_id=vocab - 1))
    else:
        raise ValueError(name)
    return m.eval()


def save_hf_model(name: str, path: str, vocab: int = 101, with_tokenizer: bool = False, seed: int = 0):
    m = make_hf_model(name, vocab, seed)
    m.save_pretrained(path, safe_serialization=True)
    if with_tokenizer:
        make_tokenizer(path, vocab)
    return m


def make_tokenizer(path: str, vocab: int):
    """Train a tiny byte-level BPE offline and save it as a HF fast tokenizer."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    corpus = ["hello world, this is a tiny corpus for an offline tokenizer."] * 50
    # deterministic alphabet that covers the corpus: ByteLevel.alphabet() is an unordered set, and a
    # corpus symbol left out of the first vocab-1 entries would get an id >= vocab
    used = sorted({c for w, _ in tok.pre_tokenizer.pre_tokenize_str(corpus[0]) for c in w})
    rest = [c for c in sorted(pre_tokenizers.ByteLevel.alphabet()) if c not in used]
    trainer = trainers.BpeTrainer(vocab_size=vocab, special_tokens=["<|endoftext|>"],
                                  initial_alphabet=(used + rest)[: vocab - 1])
    tok.train_from_iterator(corpus, trainer)
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, eos_token="<|endoftext|>", pad_token="<|endoftext|>")
    fast.save_pretrained(path)
    return fast
