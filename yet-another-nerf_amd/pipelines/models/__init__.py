from .builder import MODELS  # noqa: F401
from . import nerf_mlp, zero_outputer  # noqa: F401
