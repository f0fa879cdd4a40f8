"""Reference import path ``llmss.server.models.custom_modeling`` (``custom_modeling/__init__.py:1-7``): the
registry and the per-family classes, all over the native paged-KV decoder (``llmss_amd/models/registry.py``)."""
from llmss_amd.models.registry import CausalLM, GPT2LMHeadModel, LlamaForCausalLM, MODEL_REGISTRY  # noqa: F401

from .gpt_bigcode_modeling import GPTBigCodeForCausalLM  # noqa: F401
from .gptj_modeling import GPTJForCausalLM  # noqa: F401
