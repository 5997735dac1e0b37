"""PIL-backed stand-in for imageio.imread/imwrite (golden generator only)."""
import numpy as np
from PIL import Image


def imread(path, *args, **kwargs):
    return np.asarray(Image.open(path))


def imwrite(path, arr, *args, **kwargs):
    Image.fromarray(np.asarray(arr)).save(path)
