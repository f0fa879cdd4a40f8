"""Reference import path ``custom_modeling/gpt_bigcode_modeling.py``: ``GPTBigCodeForCausalLM`` and the module's
softmax helpers (``llmss_amd/models/family_ops.py``)."""
from llmss_amd.models.family_ops import masked_softmax, upcast_masked_softmax, upcast_softmax  # noqa: F401
from llmss_amd.models.registry import GPTBigCodeForCausalLM  # noqa: F401
