"""Per-request sampling parameters (mirrors the reference CLI/HTTP fields, generate.py:21-40,
producer_server.py:9-15) plus the deterministic per-step seed used identically on every rank.

Filter order. The reference builds HF warpers in the order TopP -> TopK -> Temperature
(generate.py:111-119) but then inverts its own test (``if not list_of_warpers``), so the warpers
are never applied: its effective sampler is plain multinomial sampling from softmax(logits) at
temperature 1 whatever the flags say. Here the flags are honoured in the order HF ``generate()``
applies them - temperature, then top-k, then top-p on the temperature-scaled distribution
(csrc/sampling.hip, ops/reference.sample) - because that is what a caller of these flags expects
and it keeps top-p's nucleus consistent with the distribution actually sampled. The reference's
*stated* order would compute the nucleus at temperature 1 and rescale afterwards; the two agree
whenever temperature == 1 (the reference's default) or when top-p == 1. The reference's *effective*
behaviour is ``temperature=1.0, top_k=0, top_p=1.0`` (unfiltered multinomial sampling), which these
parameters reproduce exactly.
"""
from __future__ import annotations

import itertools
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

_seed_counter = itertools.count(int.from_bytes(os.urandom(4), "little"))
MASK64 = (1 << 64) - 1


@dataclass
class SamplingParams:
    max_new_tokens: int = 20
    is_greedy: bool = False
    temperature: float = 1.0
    top_p: float = 0.95
    top_k: int = 50
    seed: Optional[int] = None
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False

    def validate(self) -> "SamplingParams":
        """Reference validation (generate.py:37-40)."""
        if not self.max_new_tokens > 0:
            raise ValueError("Value of max_new_tokens should be over than 0.")
        if not (0.0 < self.temperature <= 1.0):
            raise ValueError("Value of temperature is not valid.")
        if not (0.0 < self.top_p <= 1.0):
            raise ValueError("Value of top_p is not valid.")
        if not self.top_k >= 0:
            raise ValueError("Value of top_k is not valid.")
        return self

    def resolved_seed(self) -> int:
        if self.seed is None:
            self.seed = next(_seed_counter)
        return self.seed & MASK64

    # kernel-facing values
    @property
    def k_temperature(self) -> float:
        return 0.0 if self.is_greedy else float(self.temperature)

    @property
    def k_top_k(self) -> int:
        return 1 if self.is_greedy else int(self.top_k)

    @property
    def k_top_p(self) -> float:
        return float(self.top_p)


def step_seed(seed: int, step: int) -> int:
    """splitmix64(seed + step): a fresh 64-bit Philox key per (request, generated position)."""
    z = (seed + 0x9E3779B97F4A7C15 * (step + 1)) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    z = z ^ (z >> 31)
    return z - (1 << 64) if z >= (1 << 63) else z  # as signed int64


_M = [np.uint64(v) for v in (0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 1, 30, 27, 31)]


def step_seeds(seeds: np.ndarray, steps: np.ndarray) -> np.ndarray:
    """Vectorised :func:`step_seed` (uint64 seeds, int steps) -> int64 Philox keys, bit-identical."""
    golden, m1, m2, one, s30, s27, s31 = _M
    with np.errstate(over="ignore"):
        z = seeds.astype(np.uint64) + golden * (steps.astype(np.uint64) + one)
        z = (z ^ (z >> s30)) * m1
        z = (z ^ (z >> s27)) * m2
        z = z ^ (z >> s31)
    return z.view(np.int64)
