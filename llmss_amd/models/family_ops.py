"""Module-level tensor helpers of the reference's model files, for callers that import them by name.

The engine never calls these: rotary embedding runs in the QKV GEMM epilogue (``csrc/common.h``
``qkv_store_chunk``) and attention softmax inside the attention kernels. They are plain PyTorch here so a
reference user's own code that imports them keeps working (``llmss.server.models.custom_modeling.*``).

* GPT-J (``/root/reference/src/llmss/server/models/custom_modeling/gptj_modeling.py:26-47``): the sin|cos
  position table, its per-batch broadcast, and the interleaved-pair rotation. The rotation of pair
  (x[2j], x[2j+1]) by angle a is the complex product (x[2j] + i x[2j+1]) * e^{ia}, which is how it is
  computed here.
* GPTBigCode (``.../gpt_bigcode_modeling.py:49-72``): softmax with an optional upcast, scale and boolean mask.
"""
from __future__ import annotations

from typing import Optional

import torch


def create_sinusoidal_positions(num_pos: int, dim: int) -> torch.Tensor:
    """[num_pos, dim] fp32: columns [0, dim/2) are sin(p * f_j), [dim/2, dim) cos(p * f_j),
    f_j = 10000^(-2j/dim)."""
    freq = torch.pow(10000.0, -torch.arange(0, dim, 2, dtype=torch.float32) / dim)
    ang = torch.outer(torch.arange(num_pos, dtype=torch.float32), freq)
    return torch.cat((ang.sin(), ang.cos()), dim=1)


def get_embed_positions(embed_positions: torch.Tensor, position_ids: torch.Tensor) -> torch.Tensor:
    """The [num_pos, dim] table copied once per batch row: [B, num_pos, dim] on position_ids' device."""
    t = embed_positions.to(position_ids.device)
    return t.unsqueeze(0).expand(position_ids.shape[0], *t.shape).clone()


def _pairs(x: torch.Tensor) -> torch.Tensor:
    return torch.view_as_complex(x.float().unflatten(-1, (-1, 2)).contiguous())


def rotate_every_two(x: torch.Tensor) -> torch.Tensor:
    """(x[2j], x[2j+1]) -> (-x[2j+1], x[2j]) over the last dim: each pair times i."""
    return torch.view_as_real(_pairs(x) * 1j).flatten(-2).to(x.dtype)


def apply_rotary_pos_emb(tensor: torch.Tensor, sin: torch.Tensor, cos: torch.Tensor) -> torch.Tensor:
    """tensor [B, S, H, rot] (interleaved pairs), sin / cos [B, S, rot/2] -> rotated tensor in the promoted
    dtype of tensor and the tables."""
    rot = torch.complex(cos.float(), sin.float())[:, :, None, :]
    out = torch.view_as_real(_pairs(tensor) * rot).flatten(-2)
    return out.to(torch.promote_types(tensor.dtype, sin.dtype))


def _softmax(x: torch.Tensor, scale: float = 1.0, dtype: Optional[torch.dtype] = None,
             mask: Optional[torch.Tensor] = None, mask_value: Optional[torch.Tensor] = None) -> torch.Tensor:
    y = x.to(dtype) if dtype is not None else x
    if scale != 1.0:
        y = y * scale
    if mask is not None:
        y = torch.where(mask, y, mask_value)
    return torch.softmax(y, dim=-1)


def upcast_softmax(x: torch.Tensor, scale: float, softmax_dtype: torch.dtype) -> torch.Tensor:
    """softmax(x * scale) over the last dim, computed in softmax_dtype, returned in x's dtype."""
    return _softmax(x, scale, softmax_dtype).to(x.dtype)


def upcast_masked_softmax(x: torch.Tensor, mask: torch.Tensor, mask_value: torch.Tensor, scale: float,
                          softmax_dtype: torch.dtype) -> torch.Tensor:
    """As upcast_softmax, with positions where ``mask`` is False set to mask_value before the softmax."""
    return _softmax(x, scale, softmax_dtype, mask, mask_value).to(x.dtype)


def masked_softmax(x: torch.Tensor, mask: torch.Tensor, mask_value: torch.Tensor) -> torch.Tensor:
    """softmax over the last dim with positions where ``mask`` is False set to mask_value (no upcast)."""
    return _softmax(x, mask=mask, mask_value=mask_value)
