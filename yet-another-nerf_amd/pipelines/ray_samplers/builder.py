from ...utils.registry import Registry

RAY_SAMPLERS = Registry("ray_samplers")
