from ..utils.registry import Registry

DATASETS = Registry("datasets")  # reference: yanerf/dataset/builder.py
