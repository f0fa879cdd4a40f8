"""Reference import path ``llmss.server.models.utils.layers`` -> the MI355X-backed layer library."""
from llmss_amd.models.tp_layers import (FastLayerNorm, FastLinear, SuperLayer, TensorParallelColumnLinear,  # noqa: F401
                                        TensorParallelEmbedding, TensorParallelHead, TensorParallelRowLinear,
                                        get_linear, load_layer_norm, load_layer_norm_no_bias)
