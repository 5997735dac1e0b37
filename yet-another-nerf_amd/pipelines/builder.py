from ..utils.registry import Registry

PIPELINES = Registry("pipelines")
