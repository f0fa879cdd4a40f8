"""Reference import path ``llmss.server.models.utils.hub`` (``src/llmss/server/models/utils/hub.py``): hub listing,
cache lookup, file resolution (local directory, ``WEIGHTS_CACHE_OVERRIDE``, HF cache) and the retrying downloader."""
from llmss_amd.utils.checkpoint import weight_files  # noqa: F401
from llmss_amd.utils.hub import download_weights, try_to_load_from_cache, weight_hub_files  # noqa: F401
