from llmss_amd.parallel.dist import TPGroup as FakeGroup, initialize_torch_distributed  # noqa: F401
