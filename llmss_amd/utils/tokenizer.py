"""Tokenizer loading. HF tokenizers for checkpoint directories (left padding/truncation like
the reference, generate.py:46-50); a byte-level fallback for preset/random-init models."""
from __future__ import annotations

import os
from typing import List


class ByteTokenizer:
    """UTF-8 bytes <-> ids (ids >= 256 decode to nothing). Used with synthetic presets."""

    pad_token_id = 0
    eos_token_id = None

    def __init__(self, vocab_size: int = 256):
        self.vocab_size = vocab_size

    def encode(self, text: str) -> List[int]:
        return [b % self.vocab_size for b in text.encode("utf-8")] or [0]

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        return bytes(int(i) for i in ids if 0 <= int(i) < 256).decode("utf-8", errors="replace")

    def batch_decode(self, seqs, **kw):
        return [self.decode(s) for s in seqs]


def load_tokenizer(path: str, vocab_size: int = 256):
    if os.path.isdir(path):
        try:
            from transformers import AutoTokenizer

            tok = AutoTokenizer.from_pretrained(path, padding_side="left", truncation_side="left")
            return tok
        except Exception:  # no tokenizer files in the checkpoint dir
            pass
    return ByteTokenizer(vocab_size)


def encode(tok, text: str) -> List[int]:
    if isinstance(tok, ByteTokenizer):
        return tok.encode(text)
    return tok(text, return_attention_mask=False)["input_ids"]
