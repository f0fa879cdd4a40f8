"""Reference import path ``custom_modeling/gptj_modeling.py``: ``GPTJForCausalLM`` and the module's rotary
helpers (``llmss_amd/models/family_ops.py``)."""
from llmss_amd.models.family_ops import (apply_rotary_pos_emb, create_sinusoidal_positions,  # noqa: F401
                                         get_embed_positions, rotate_every_two)
from llmss_amd.models.registry import GPTJForCausalLM  # noqa: F401
