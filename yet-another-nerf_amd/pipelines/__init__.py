"""Registry-compatible mirror of the reference's yanerf.pipelines package (same registry names, classes and
constructor/forward signatures), backed by the HIP hot path."""
from .builder import PIPELINES  # noqa: F401
from . import nerf_pipeline  # noqa: F401
