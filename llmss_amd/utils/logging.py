"""Structured logging (reference used loguru in ``hub.py``/``dist.py``; stdlib here)."""
from __future__ import annotations

import logging
import os
import sys

_CONFIGURED = False


def _configure():
    global _CONFIGURED
    if _CONFIGURED:
        return
    level = os.environ.get("LLMSS_LOG_LEVEL", "WARNING").upper()
    h = logging.StreamHandler(sys.stderr)
    rank = os.environ.get("RANK", "0")
    h.setFormatter(logging.Formatter(f"%(asctime)s [r{rank}] %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger("llmss_amd")
    root.addHandler(h)
    root.setLevel(level)
    root.propagate = False
    _CONFIGURED = True


def get_logger(name: str) -> logging.Logger:
    _configure()
    if not name.startswith("llmss_amd"):
        name = "llmss_amd." + name
    return logging.getLogger(name)
