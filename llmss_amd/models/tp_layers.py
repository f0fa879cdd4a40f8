"""Reference-compatible tensor-parallel layer API, backed by the gfx950 kernels.

Reference: ``src/llmss/server/models/utils/layers.py`` - ``FastLinear`` / ``get_linear`` /
``SuperLayer`` (``:39-76``), ``TensorParallelHead`` (``:79-135``), ``TensorParallelColumnLinear``
(``:138-153``), ``TensorParallelRowLinear`` (``:156-179``), ``TensorParallelEmbedding``
(``:182-214``), ``nn.LayerNorm.load`` / ``load_no_bias`` (``:12-36``) and the optional fused
``FastLayerNorm`` (``:217-253``), all over ``Weights`` (``utils/weights.py:9-115``).

The serving engine does not build models out of these modules (``DecoderLM`` fuses QKV and
gate/up at load time and drives the kernels directly); they exist so code written against the
reference's layer library runs unchanged on MI355X:

* every linear is the hand-written MFMA GEMM (``ops.linear``; PyTorch only for CPU tensors);
* the row-parallel all-reduce and the head all-gather go through the TP communicator (RCCL on GPU);
* ``TensorParallelHead`` pads the vocabulary to a multiple of the TP degree and shards it (the
  reference replicates the whole head when ``V % tp != 0``) and trims the gathered logits back to V;
* ``TensorParallelEmbedding`` keeps the full table on every rank, so ``reduce=True`` needs no
  all-reduce at all; ``reduce=False`` returns the rank's vocab-slice lookup like the reference;
* ``FastLayerNorm`` is the fused residual-add + LayerNorm kernel and is the class
  ``nn.LayerNorm.load`` returns, so it is on the hot path (the reference defines it but never uses it).
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn

from .. import ops
from ..parallel.dist import TPGroup, as_tp_group


class ProcessGroupView:
    """``size()`` / ``rank()`` view of a :class:`TPGroup`, a reference ``FakeGroup`` or a torch ProcessGroup -
    the interface the reference layer code calls (``weights.process_group.size()``), plus the two collectives
    it needs. Every kind maps to a TPGroup (parallel/dist.py as_tp_group)."""

    def __init__(self, group=None):
        self.tp = as_tp_group(group)

    def size(self) -> int:
        return self.tp.size

    def rank(self) -> int:
        return self.tp.rank

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        return self.tp.all_reduce(t)

    def all_gather_last_dim(self, t: torch.Tensor) -> torch.Tensor:
        return self.tp.all_gather_last_dim(t)


def as_group_view(group) -> ProcessGroupView:
    return group if isinstance(group, ProcessGroupView) else ProcessGroupView(group)


def _linear2d(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if x2.is_cuda and x2.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and shp[-1] % 16 == 0:
        y = ops.linear(x2.contiguous(), weight, bias)
    else:  # CPU tensors / dtypes the MFMA kernels do not take
        y = torch.nn.functional.linear(x2, weight, bias)
    return y.reshape(*shp[:-1], weight.shape[0])


class FastLinear(nn.Module):
    def __init__(self, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> None:
        super().__init__()
        self.weight = nn.Parameter(weight.contiguous(), requires_grad=False)
        self.bias = nn.Parameter(bias.contiguous(), requires_grad=False) if bias is not None else None

    @classmethod
    def load(cls, config, prefix: str, weights, bias: bool):
        w = weights.get_tensor(f"{prefix}.weight")
        b = weights.get_tensor(f"{prefix}.bias") if bias else None
        return cls(w, b)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _linear2d(x, self.weight, self.bias)


def get_linear(weight, bias):
    return FastLinear(weight, bias)


class SuperLayer(nn.Module):
    def __init__(self, linear):
        super().__init__()
        self.linear = linear

    def forward(self, x):
        return self.linear.forward(x)


class TensorParallelHead(SuperLayer):
    def __init__(self, linear, process_group, should_gather: bool, vocab_size: Optional[int] = None):
        super().__init__(linear)
        self.process_group = as_group_view(process_group)
        self.should_gather = should_gather
        self.vocab_size = vocab_size

    @staticmethod
    def load(config, prefix: str, weights):
        pg = as_group_view(weights.process_group)
        V = weights.get_shape(f"{prefix}.weight")[0]
        if pg.size() == 1:
            return TensorParallelHead(get_linear(weights.get_tensor(f"{prefix}.weight"), None), pg, False, V)
        vl = -(-V // pg.size())  # pad the vocab instead of replicating the head (reference :91-95)
        lo = pg.rank() * vl
        full = weights.get_tensor(f"{prefix}.weight") if lo < V else None
        w = torch.zeros(vl, weights.get_shape(f"{prefix}.weight")[1], dtype=weights.dtype, device=weights.device)
        if full is not None:
            n = min(V, lo + vl) - lo
            w[:n] = full[lo:lo + n]
        return TensorParallelHead(get_linear(w, None), pg, True, V)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = super().forward(x)
        if self.should_gather:
            out = self.process_group.all_gather_last_dim(out)
        if self.vocab_size is not None and out.shape[-1] != self.vocab_size:
            out = out[..., :self.vocab_size]
        return out


class TensorParallelColumnLinear(SuperLayer):
    @classmethod
    def load(cls, config, prefix: str, weights, bias: bool):
        return cls.load_multi(config, [prefix], weights, bias, dim=0)

    @classmethod
    def load_multi(cls, config, prefixes: List[str], weights, bias: bool, dim: int):
        weight = weights.get_multi_weights_col(prefixes, dim=dim)
        b = torch.cat([weights.get_sharded(f"{p}.bias", dim=0) for p in prefixes], dim=dim) if bias else None
        return cls(get_linear(weight, b))


class TensorParallelRowLinear(SuperLayer):
    def __init__(self, linear, process_group):
        super().__init__(linear)
        self.process_group = as_group_view(process_group)

    @classmethod
    def load(cls, config, prefix: str, weights, bias: bool):
        pg = as_group_view(weights.process_group)
        weight = weights.get_multi_weights_row(prefix)
        b = weights.get_tensor(f"{prefix}.bias") if bias and pg.rank() == 0 else None  # added once by the reduce
        return cls(get_linear(weight, b), process_group=pg)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = super().forward(x)
        if self.process_group.size() > 1:
            self.process_group.all_reduce(out)
        return out


class TensorParallelEmbedding(nn.Module):
    def __init__(self, prefix: str, weights, reduce: bool = True):
        super().__init__()
        pg = as_group_view(weights.process_group)
        self.process_group = pg
        self.reduce = reduce
        full = weights.get_tensor(f"{prefix}.weight")
        V = full.shape[0]
        block = -(-V // pg.size())  # every id has an owner, also when V % tp != 0 (reference quirk Q6)
        self.min_id = pg.rank() * block
        self.max_id = min(V, self.min_id + block)
        self.weight = nn.Parameter(full, requires_grad=False)  # replicated: lookups need no all-reduce

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if self.reduce or self.process_group.size() == 1:
            flat = ids.reshape(-1)
            if self.weight.is_cuda and self.weight.dtype == torch.bfloat16:
                out = ops.embed(flat.to(torch.int64).contiguous(), self.weight)
            else:
                out = torch.nn.functional.embedding(flat, self.weight)
            return out.reshape(*ids.shape, self.weight.shape[1])
        own = (ids >= self.min_id) & (ids < self.max_id)  # reduce=False: this rank's vocab slice only
        out = torch.nn.functional.embedding(ids.clamp(0, self.weight.shape[0] - 1), self.weight)
        return out * own.unsqueeze(-1).to(out.dtype)


class FastLayerNorm(nn.LayerNorm):
    """LayerNorm (or RMSNorm when there is no bias and ``rms``) with the residual add fused:
    ``forward(h, residual) -> (normed, h + residual)`` on the add_norm kernel (reference ``:220-253``)."""

    rms = False

    def forward(self, hidden_states, residual=None):
        if hidden_states.is_cuda and hidden_states.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16:
            shp = hidden_states.shape
            h2 = hidden_states.reshape(-1, shp[-1]).contiguous()
            r2 = residual.reshape(-1, shp[-1]).contiguous().clone() if residual is not None else None
            y, r = ops.add_norm(h2, self.weight, self.bias, self.eps, self.rms, r2)
            return y.reshape(shp), r.reshape(shp)
        if residual is not None:
            hidden_states = hidden_states + residual
        residual = hidden_states
        if self.rms:
            x = hidden_states.float()
            y = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps)).to(hidden_states.dtype) * self.weight
        else:
            y = super().forward(hidden_states)
        return y, residual


def load_layer_norm(cls, prefix: str, weights, eps: float):
    w = weights.get_tensor(f"{prefix}.weight")
    b = weights.get_tensor(f"{prefix}.bias")
    ln = FastLayerNorm(w.shape[0], eps=eps, device="meta")
    ln.weight = nn.Parameter(w, requires_grad=False)
    ln.bias = nn.Parameter(b, requires_grad=False)
    return ln


def load_layer_norm_no_bias(cls, prefix: str, weights, eps: float):
    w = weights.get_tensor(f"{prefix}.weight")
    ln = FastLayerNorm(w.shape[0], eps=eps, device="meta")
    ln.weight = nn.Parameter(w, requires_grad=False)
    ln.bias = None
    ln.rms = True  # bias-free norms in the target families are RMSNorm (Llama)
    return ln


# reference API: torch.nn.LayerNorm.load(prefix=..., weights=..., eps=...) (layers.py:35-36)
torch.nn.LayerNorm.load = classmethod(load_layer_norm)
torch.nn.LayerNorm.load_no_bias = classmethod(load_layer_norm_no_bias)
