from .builder import FEATURE_EXTRACTORS  # noqa: F401
from . import identity_mapper  # noqa: F401
