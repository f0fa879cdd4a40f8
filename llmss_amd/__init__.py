"""llmss_amd - MI355X-native (gfx950 / CDNA4) tensor-parallel LLM serving.

Capabilities of jongwon-jay-lee/llmss (tensor-parallel GPT-J / GPT-BigCode inference, the
``generate.py`` CLI and the FastAPI -> Redis -> torchrun pub/sub server), rebuilt around
hand-written HIP kernels for gfx950, RCCL over xGMI, HIP-graph-captured decode and a C++
runtime; extended with GPT-2, Llama-2 (RMSNorm, SwiGLU, GQA), fp8 weights and a gRPC API.
"""
import torch  # noqa: F401  (load torch's HIP runtime before our extension shares it)

__version__ = "0.1.0"

_NATIVE = None


def _native():
    """The compiled native module (kernels + runtime). Builds it in-tree on first use if absent."""
    global _NATIVE
    if _NATIVE is None:
        try:
            from . import _C
        except ImportError:
            from . import _build

            _build.build()
            from . import _C
        _NATIVE = _C
    return _NATIVE
