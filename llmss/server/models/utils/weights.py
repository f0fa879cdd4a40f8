from llmss_amd.models.registry import Weights  # noqa: F401
