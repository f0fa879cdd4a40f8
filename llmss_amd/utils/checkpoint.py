"""Checkpoint file resolution and sharded tensor reads.

Reference: ``utils/hub.py`` (weight_files / HF cache resolution, ``hub.py:19-118``) and
``utils/weights.py`` (safetensors routing table + ``get_partial_sharded`` slicing,
``weights.py:9-115``). Here the reads go through the native ``SafetensorsFile`` (C++ mmap,
multi-threaded slice copies, only the shard's bytes are touched) into torch CPU tensors;
``.bin`` checkpoints are read with ``torch.load(weights_only=True)`` (never unpickling code).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional

import torch

from .logging import get_logger

log = get_logger(__name__)

_ST_DTYPES = {
    "F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
    "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
    "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn, "F8_E5M2": torch.float8_e5m2,
}


def weight_files(model_path: str, extension: str = ".safetensors") -> List[str]:
    """Local directory -> sorted weight files (hub.py:77-118 minus network access).

    ``WEIGHTS_CACHE_OVERRIDE`` (hub.py:16,98-105) and the HF cache snapshot layout are honoured.
    """
    override = os.environ.get("WEIGHTS_CACHE_OVERRIDE")
    cands = []
    if override:
        cands.append(os.path.join(override, model_path.replace("/", "--")))
        cands.append(override)
    cands.append(model_path)
    hub = os.environ.get("HUGGINGFACE_HUB_CACHE") or os.environ.get("HF_HUB_CACHE")
    if hub:
        snap = glob.glob(os.path.join(hub, "models--" + model_path.replace("/", "--"), "snapshots", "*"))
        cands.extend(sorted(snap))
    for d in cands:
        if os.path.isdir(d):
            files = sorted(glob.glob(os.path.join(d, f"*{extension}")))
            files = [f for f in files if not any(s in os.path.basename(f) for s in ("arguments", "args", "training"))]
            if files:
                return files
            if extension == ".safetensors":
                bins = sorted(glob.glob(os.path.join(d, "*.bin")))
                bins = [f for f in bins if not any(s in os.path.basename(f) for s in ("arguments", "args", "training"))]
                if bins:
                    return bins
    raise FileNotFoundError(f"no weight files found for {model_path!r}")


class CheckpointReader:
    """Name -> file routing over one or more checkpoint files with sharded reads."""

    def __init__(self, files: List[str], aliases: Optional[Dict[str, List[str]]] = None, threads: int = 8):
        from .. import _native

        self.threads = threads
        self._st = {}
        self._bin = {}
        self.routing: Dict[str, str] = {}
        self.aliases = aliases or {}
        for f in files:
            if f.endswith(".safetensors"):
                h = _native().SafetensorsFile(f)
                self._st[f] = h
                keys = h.keys()
            else:
                sd = torch.load(f, map_location="cpu", weights_only=True, mmap=True)
                self._bin[f] = sd
                keys = list(sd.keys())
            for k in keys:
                if k in self.routing:
                    raise RuntimeError(f"tensor {k} found in multiple files: {f} and {self.routing[k]}")
                self.routing[k] = f

    def metadata(self) -> Dict[str, str]:
        """Merged ``__metadata__`` of the safetensors files."""
        out: Dict[str, str] = {}
        for h in self._st.values():
            out.update(h.metadata())
        return out

    # ------------------------------------------------------------------ lookup
    def resolve(self, name: str) -> str:
        if name in self.routing:
            return name
        for a in self.aliases.get(name, []):
            if a in self.routing:
                return a
        raise KeyError(f"weight {name} does not exist")

    def has(self, name: str) -> bool:
        try:
            self.resolve(name)
            return True
        except KeyError:
            return False

    def find(self, *names: str) -> Optional[str]:
        for n in names:
            if self.has(n):
                return self.resolve(n)
        return None

    def shape(self, name: str) -> List[int]:
        name = self.resolve(name)
        f = self.routing[name]
        if f in self._st:
            return list(self._st[f].info(name)[1])
        return list(self._bin[f][name].shape)

    def keys(self) -> List[str]:
        return list(self.routing)

    # ------------------------------------------------------------------ reads
    def get(self, name: str, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        shp = self.shape(name)
        return self.slice(name, 0, 0, shp[0] if shp else 1, dtype)

    def slice(self, name: str, dim: int, start: int, stop: int, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        name = self.resolve(name)
        f = self.routing[name]
        if f in self._bin:
            t = self._bin[f][name]
            t = t.narrow(dim, start, stop - start).contiguous() if t.dim() else t.clone()
        else:
            h = self._st[f]
            dt, shp, _, _ = h.info(name)
            tdt = _ST_DTYPES[dt]
            shp = list(shp)
            if shp:
                shp[dim] = stop - start
            t = torch.empty(shp, dtype=tdt)
            if t.numel():
                h.copy_slice(name, dim, start, stop, t.data_ptr(), self.threads)
        if dtype is not None and t.is_floating_point() and t.dtype != dtype:
            t = t.to(dtype)
        return t

    def rows(self, name, start, stop, dtype=None):
        return self.slice(name, 0, start, stop, dtype)

    def cols(self, name, start, stop, dtype=None):
        return self.slice(name, 1, start, stop, dtype)
