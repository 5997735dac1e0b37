from ...utils.registry import Registry

FEATURE_EXTRACTORS = Registry("feature_extractors")
