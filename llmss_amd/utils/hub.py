"""Hugging Face hub resolution + downloader (reference ``utils/hub.py``).

* :func:`weight_hub_files` - list a hub repo's weight files, dropping training/argument
  artefacts (hub.py:19-39).
* :func:`try_to_load_from_cache` / :func:`weight_files_resolved` - local dir -> HF cache snapshot ->
  hub listing (hub.py:42-118); local resolution lives in :func:`checkpoint.weight_files`.
* :func:`download_weights` - per-file download with bounded retries and backoff, logging duration
  and an ETA (hub.py:121-163; the reference never calls it, here ``generate.py --download`` does).

Network access is optional: with ``HF_HUB_OFFLINE=1`` (or no ``huggingface_hub``) every call resolves
from local files only and raises ``FileNotFoundError`` when nothing is there.
"""
from __future__ import annotations

import os
import time
from datetime import timedelta
from pathlib import Path
from typing import Callable, List, Optional

from .checkpoint import weight_files
from .logging import get_logger

log = get_logger(__name__)

_SKIP = ("arguments", "args", "training")


def _offline() -> bool:
    return os.environ.get("HF_HUB_OFFLINE", "0") not in ("0", "", "false", "False")


def _filter(names: List[str], extension: str) -> List[str]:
    return sorted(n for n in names if n.endswith(extension) and not any(s in Path(n).name for s in _SKIP))


def weight_hub_files(model_id: str, revision: Optional[str] = None, extension: str = ".safetensors",
                     list_files: Optional[Callable[..., List[str]]] = None) -> List[str]:
    """Weight file names of a hub repo (no download)."""
    if list_files is None:
        if _offline():
            raise FileNotFoundError(f"HF_HUB_OFFLINE=1: cannot list {model_id}")
        from huggingface_hub import list_repo_files

        list_files = list_repo_files
    names = _filter(list(list_files(model_id, revision=revision)), extension)
    if not names and extension == ".safetensors":
        names = _filter(list(list_files(model_id, revision=revision)), ".bin")
    if not names:
        raise FileNotFoundError(f"no {extension} weights in {model_id}")
    return names


def try_to_load_from_cache(model_id: str, revision: Optional[str], filename: str) -> Optional[Path]:
    """Path of ``filename`` in the local HF cache snapshot, or None."""
    hub = os.environ.get("HUGGINGFACE_HUB_CACHE") or os.environ.get("HF_HUB_CACHE")
    if not hub:
        hub = os.path.join(os.path.expanduser("~"), ".cache", "huggingface", "hub")
    repo = Path(hub) / ("models--" + model_id.replace("/", "--"))
    if not repo.is_dir():
        return None
    snap = None
    if revision is not None and (repo / "snapshots" / revision).is_dir():
        snap = repo / "snapshots" / revision
    else:
        ref = repo / "refs" / (revision or "main")
        if ref.is_file():
            snap = repo / "snapshots" / ref.read_text().strip()
    if snap is None:
        snaps = sorted((repo / "snapshots").glob("*")) if (repo / "snapshots").is_dir() else []
        snap = snaps[-1] if snaps else None
    if snap is None:
        return None
    p = snap / filename
    return p if p.exists() else None


def weight_files_resolved(model_id: str, revision: Optional[str] = None, extension: str = ".safetensors",
                          download: bool = False) -> List[str]:
    """Local dir / cache first; optionally download what is missing."""
    try:
        return weight_files(model_id, extension)
    except FileNotFoundError:
        if not download:
            raise
    names = weight_hub_files(model_id, revision, extension)
    return [str(p) for p in download_weights(names, model_id, revision)]


def download_weights(filenames: List[str], model_id: str, revision: Optional[str] = None, tries: int = 5,
                     backoff_s: float = 5.0, fetch: Optional[Callable[..., str]] = None) -> List[Path]:
    """Fetch ``filenames`` (cache hits are free); each file is retried ``tries`` times."""
    if fetch is None:
        if _offline():
            raise FileNotFoundError(f"HF_HUB_OFFLINE=1: cannot download {model_id}")
        from huggingface_hub import hf_hub_download

        fetch = hf_hub_download
    out: List[Path] = []
    t_start = time.time()
    for i, name in enumerate(filenames):
        cached = try_to_load_from_cache(model_id, revision, name)
        if cached is not None:
            out.append(cached)
            continue
        t0 = time.time()
        for attempt in range(1, tries + 1):
            try:
                p = fetch(repo_id=model_id, filename=name, revision=revision)
                break
            except Exception as e:  # network errors of every flavour: retry, then surface the last one
                if attempt == tries:
                    raise
                log.warning("download %s failed (%s), retry %d/%d in %.0fs", name, e, attempt, tries - 1, backoff_s)
                time.sleep(backoff_s)
        out.append(Path(p))
        done = i + 1
        eta = (time.time() - t_start) / done * (len(filenames) - done)
        log.info("downloaded %s in %s (%d/%d, ETA %s)", name, timedelta(seconds=int(time.time() - t0)), done,
                 len(filenames), timedelta(seconds=int(eta)))
    return out
