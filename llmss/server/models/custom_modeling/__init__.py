from llmss_amd.models.registry import MODEL_REGISTRY, CausalLM  # noqa: F401
