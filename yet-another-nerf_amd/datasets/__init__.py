"""Data side of the training path (reference yanerf/dataset): Blender (nerf_synthetic) and LLFF loaders under the
same registry names, constructor arguments and item layout, plus DeviceImageSet, which keeps a whole split resident
in HBM so a training step never copies an image host-to-device."""
from .blender_dataset import BlenderDataset, BlenderDatasetWrapper
from .builder import DATASETS
from .device_set import DeviceImageSet
from .llff_dataset import LLFFDataset, LLFFDatasetWrapper

__all__ = ["DATASETS", "BlenderDataset", "BlenderDatasetWrapper", "LLFFDataset", "LLFFDatasetWrapper",
           "DeviceImageSet"]
