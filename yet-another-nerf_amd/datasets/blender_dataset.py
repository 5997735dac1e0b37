"""nerf_synthetic (Blender) loader, reference yanerf/dataset/blender_dataset.py:24-78."""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Callable, NamedTuple, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .builder import DATASETS
from .utils import load_image, resize_linear

logger = logging.getLogger(__name__)


class BlenderDatasetWrapper(NamedTuple):
    poses: torch.Tensor
    focal_lengths: torch.Tensor
    image_rgb: torch.Tensor


@DATASETS.register_module()
class BlenderDataset(Dataset):
    """Items are (pose [3|4,4] c2w with the camera-axis flip diag(1,-1,-1,1), focal [1], image [H,W,3] in [0,1]).

    Same arguments and quirks as the reference:
      * val/test keep every `test_skip`-th frame (:36-38);
      * focal = 0.5 W / tan(0.5 camera_angle_x) from the FIRST frame's image size (:41-44), divided by scale_down;
      * `debug` forces scale_down = 32 (:46-48); H, W = floor division (:52-53);
      * the resized image has shape (W // s, H // s): the reference passes dsize=(H, W) to cv2.resize, whose dsize is
        (width, height) (:69) -- identical for the square nerf_synthetic images.
    """
    data_wrapper: Callable = BlenderDatasetWrapper

    def __init__(self, base_dir, split, scale_down=1, test_skip=8, debug=False):
        if split not in ["train", "val", "test"]:
            raise ValueError(f"Invalid split: {split}.")
        self.base_dir = Path(base_dir)
        self.split = split
        with open(self.base_dir / f"transforms_{split}.json", "r") as fp:
            meta = json.load(fp)
        self.frames = meta["frames"]
        if split in ["val", "test"]:
            self.frames = self.frames[::test_skip]
        camera_angle_x = float(meta["camera_angle_x"])
        img = load_image(self.base_dir / f"{self.frames[0]['file_path']}.png")
        H, W = img.shape[:2]
        focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
        if debug:
            scale_down = 32
        if scale_down < 0 or not isinstance(scale_down, (float, int)):
            raise TypeError(f"Invalid type scale_down: {type(scale_down)}.")
        self.H = H // scale_down
        self.W = W // scale_down
        self.focal = focal / scale_down
        self.scale_down = scale_down
        calib = np.eye(4).astype(np.float32)
        calib[1, 1] = calib[2, 2] = -1.0
        self.calib_mat = calib

    def __getitem__(self, index: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        frame = self.frames[index]
        pose = np.array(frame["transform_matrix"]).astype(np.float32) @ self.calib_mat  # (:60-64)
        img = load_image(self.base_dir / f"{frame['file_path']}.png")
        if self.scale_down != 1:
            img = resize_linear(img, self.W, self.H)  # cv2 dsize=(H, W) means width H, height W
        return torch.from_numpy(pose), torch.FloatTensor([self.focal]), torch.from_numpy(img)

    def __len__(self):
        return len(self.frames)
