from ...utils.registry import Registry

RENDERERS = Registry("renderers")
