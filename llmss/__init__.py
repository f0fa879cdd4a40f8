"""Import-compatible façade for code written against the reference package layout
(``llmss.server.models.custom_modeling.MODEL_REGISTRY``, ``llmss.server.models.utils.*``).
Everything resolves to the MI355X-native implementation in :mod:`llmss_amd`."""
