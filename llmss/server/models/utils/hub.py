from llmss_amd.utils.checkpoint import weight_files  # noqa: F401
