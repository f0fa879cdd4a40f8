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


_TOKENIZER_FILES = ("tokenizer.json", "tokenizer_config.json", "vocab.json", "merges.txt", "tokenizer.model",
                    "spiece.model", "vocab.txt")


def load_tokenizer(path: str, vocab_size: int = 256):
    """HF tokenizer of a checkpoint directory; the byte tokenizer ONLY for synthetic presets and
    checkpoint directories that ship no tokenizer files (logged). A directory whose tokenizer files
    exist but fail to load raises: silently decoding garbage through the byte fallback would hide it."""
    from .logging import get_logger

    if os.path.isdir(path):
        present = [f for f in _TOKENIZER_FILES if os.path.exists(os.path.join(path, f))]
        if present:
            from transformers import AutoTokenizer

            try:
                return AutoTokenizer.from_pretrained(path, padding_side="left", truncation_side="left")
            except Exception as e:
                raise RuntimeError(f"tokenizer files {present} in {path} could not be loaded: {e}") from e
        get_logger(__name__).warning("%s has no tokenizer files: using the byte-level tokenizer", path)
    return ByteTokenizer(vocab_size)


def encode(tok, text: str) -> List[int]:
    if isinstance(tok, ByteTokenizer):
        return tok.encode(text)
    return tok(text, return_attention_mask=False)["input_ids"]


class StreamDecoder:
    """Incremental detokenisation of a token stream: each new token costs one decode of a short window
    (the tokens since the last emitted text boundary, a few ids) instead of decoding the whole sequence
    again - O(n) per request instead of O(n^2). Text is held back while the window ends inside a
    multi-byte / multi-token character (decode yields U+FFFD), so the concatenated pieces equal
    ``tok.decode(all_ids)``."""

    def __init__(self, tok):
        self.tok = tok
        self.ids: List[int] = []
        self.prefix = 0  # window start (ids before it are already emitted text)
        self.read = 0  # ids [prefix, read) decode to text that has been emitted

    def push(self, token_id: int) -> str:
        self.ids.append(int(token_id))
        emitted = self.tok.decode(self.ids[self.prefix:self.read])
        full = self.tok.decode(self.ids[self.prefix:])
        if len(full) > len(emitted) and not full.endswith("\ufffd"):
            self.prefix, self.read = self.read, len(self.ids)
            return full[len(emitted):]
        return ""

    def flush(self) -> str:
        """Whatever is still held back (a stream that ends inside a character)."""
        emitted = self.tok.decode(self.ids[self.prefix:self.read])
        full = self.tok.decode(self.ids[self.prefix:])
        self.prefix = self.read = len(self.ids)
        return full[len(emitted):]
