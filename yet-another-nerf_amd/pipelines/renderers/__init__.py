from .builder import RENDERERS  # noqa: F401
from . import multipass_emission_absorpsion_renderer  # noqa: F401
