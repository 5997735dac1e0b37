from ...utils.registry import Registry

MODELS = Registry("models")
