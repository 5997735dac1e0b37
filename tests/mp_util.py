"""Result passing for the multi-process tests."""
import numpy as np
import torch


def _by_value(obj):
    """Tensors as numpy arrays for the result queue: torch's queue pickling shares a CPU tensor's storage through a
    file descriptor served by the sending process, which fails once that process has exited before the parent
    unpickles (seen on a GPU box: FileNotFoundError in resource_sharer)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_by_value(x) for x in obj)
    if isinstance(obj, dict):
        return {k: _by_value(v) for k, v in obj.items()}
    return obj


def _as_tensors(obj):
    if isinstance(obj, np.ndarray):
        return torch.from_numpy(obj)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_as_tensors(x) for x in obj)
    if isinstance(obj, dict):
        return {k: _as_tensors(v) for k, v in obj.items()}
    return obj
