"""Reference import path ``llmss.server.models.utils.dist`` (``src/llmss/server/models/utils/dist.py``): the
reference's ``FakeBarrier`` / ``FakeGroup`` API and ``initialize_torch_distributed`` over the native runtime."""
from llmss_amd.parallel.dist import FakeBarrier, FakeGroup, as_tp_group, initialize_torch_distributed  # noqa: F401
