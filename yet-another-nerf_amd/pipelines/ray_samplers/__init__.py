from .builder import RAY_SAMPLERS  # noqa: F401
from . import ray_sampler  # noqa: F401
from .utils import EvaluationMode, RayBundle, RenderSamplingMode, get_xy_grid  # noqa: F401
