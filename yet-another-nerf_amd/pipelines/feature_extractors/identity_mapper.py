"""IdentityMapper: passes its kwargs through (reference feature_extractors/identity_mapper.py:6-11)."""
import torch

from .builder import FEATURE_EXTRACTORS


@FEATURE_EXTRACTORS.register_module()
class IdentityMapper(torch.nn.Module):
    def forward(self, **kwargs):
        return kwargs
