"""LLFF (forward-facing, e.g. Fern) loader, reference yanerf/dataset/llff_dataset.py:26-382.

The pose arithmetic (axis reorder, bound rescale, recentering, spiral / spherified render paths, hold-out split) is
restated step for step in float math identical to the reference's numpy code; items carry the per-image near/far
bounds the ray sampler consumes (ray_sampler.py:280-283)."""
from __future__ import annotations

import logging
import os
from typing import Callable, NamedTuple, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from .builder import DATASETS
from .utils import load_image

logger = logging.getLogger(__name__)
_IMG_EXT = ("JPG", "jpg", "png")


class LLFFDatasetWrapper(NamedTuple):
    poses: torch.Tensor
    focal_lengths: torch.Tensor
    image_rgb: torch.Tensor
    min_depth: torch.Tensor
    max_depth: torch.Tensor


def normalize(x):
    return x / np.linalg.norm(x)


def viewmatrix(z, up, pos):
    """Camera-to-world [3,4] looking along z with the given up vector (llff_dataset.py:278-284)."""
    vec2 = normalize(z)
    vec0 = normalize(np.cross(up, vec2))
    vec1 = normalize(np.cross(vec2, vec0))
    return np.stack([vec0, vec1, vec2, pos], 1)


def poses_avg(poses):
    """Mean camera [3,5] (with the first pose's hwf column) (llff_dataset.py:292-301)."""
    hwf = poses[0, :3, -1:]
    center = poses[:, :3, 3].mean(0)
    vec2 = normalize(poses[:, :3, 2].sum(0))
    up = poses[:, :3, 1].sum(0)
    return np.concatenate([viewmatrix(vec2, up, center), hwf], 1)


def render_path_spiral(c2w, up, rads, focal, zdelta, zrate, rots, N):
    """Spiral of N cameras around c2w focusing at depth `focal` (llff_dataset.py:304-313)."""
    out = []
    rads = np.array(list(rads) + [1.0])
    hwf = c2w[:, 4:5]
    for theta in np.linspace(0.0, 2.0 * np.pi * rots, int(N) + 1)[:-1]:
        c = np.dot(c2w[:3, :4], np.array([np.cos(theta), -np.sin(theta), -np.sin(theta * zrate), 1.0]) * rads)
        z = normalize(c - np.dot(c2w[:3, :4], np.array([0, 0, -focal, 1.0])))
        out.append(np.concatenate([viewmatrix(z, up, c), hwf], 1))
    return out


def recenter_poses(poses):
    """Express every pose in the frame of the average pose (llff_dataset.py:316-328)."""
    out = poses + 0
    bottom = np.reshape([0, 0, 0, 1.0], [1, 4])
    c2w = np.concatenate([poses_avg(poses)[:3, :4], bottom], -2)
    bottom = np.tile(np.reshape(bottom, [1, 1, 4]), [poses.shape[0], 1, 1])
    p = np.concatenate([poses[:, :3, :4], bottom], -2)
    p = np.linalg.inv(c2w) @ p
    out[:, :3, :4] = p[:, :3, :4]
    return out


def spherify_poses(poses, bds):
    """Recentre on the rays' closest point, normalise the radius, and build a 120-view circle
    (llff_dataset.py:334-382). Returns (poses_reset [N,3,5], render_poses [120,3,5], bds)."""
    def p34_to_44(p):
        return np.concatenate([p, np.tile(np.reshape(np.eye(4)[-1, :], [1, 1, 4]), [p.shape[0], 1, 1])], 1)

    rays_d = poses[:, :3, 2:3]
    rays_o = poses[:, :3, 3:4]
    A_i = np.eye(3) - rays_d * np.transpose(rays_d, [0, 2, 1])
    b_i = -A_i @ rays_o
    center = np.squeeze(-np.linalg.inv((np.transpose(A_i, [0, 2, 1]) @ A_i).mean(0)) @ b_i.mean(0))
    up = (poses[:, :3, 3] - center).mean(0)
    vec0 = normalize(up)
    vec1 = normalize(np.cross([0.1, 0.2, 0.3], vec0))
    vec2 = normalize(np.cross(vec0, vec1))
    c2w = np.stack([vec1, vec2, vec0, center], 1)
    poses_reset = np.linalg.inv(p34_to_44(c2w[None])) @ p34_to_44(poses[:, :3, :4])
    rad = np.sqrt(np.mean(np.sum(np.square(poses_reset[:, :3, 3]), -1)))
    sc = 1.0 / rad
    poses_reset[:, :3, 3] *= sc
    bds *= sc
    rad *= sc
    centroid = np.mean(poses_reset[:, :3, 3], 0)
    zh = centroid[2]
    radcircle = np.sqrt(rad ** 2 - zh ** 2)
    new_poses = []
    for th in np.linspace(0.0, 2.0 * np.pi, 120):
        camorigin = np.array([radcircle * np.cos(th), radcircle * np.sin(th), zh])
        upv = np.array([0, 0, -1.0])
        v2 = normalize(camorigin)
        v0 = normalize(np.cross(v2, upv))
        v1 = normalize(np.cross(v2, v0))
        new_poses.append(np.stack([v0, v1, v2, camorigin], 1))
    new_poses = np.stack(new_poses, 0)
    new_poses = np.concatenate([new_poses, np.broadcast_to(poses[0, :3, -1:], new_poses[:, :3, -1:].shape)], -1)
    poses_reset = np.concatenate(
        [poses_reset[:, :3, :4], np.broadcast_to(poses[0, :3, -1:], poses_reset[:, :3, -1:].shape)], -1)
    return poses_reset, new_poses, bds


def _list_images(d):
    return [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(_IMG_EXT)]


def load_llff_data(basedir, factor=None, width=None, height=None):
    """poses [3,5,N] (rotation | translation | hwf), bds [2,N], image files (llff_dataset.py:160-210).

    The reference creates a missing `images_<factor>` / `images_<W>x<H>` directory by shelling out to ImageMagick
    `mogrify` (:212-258). That external tool is not part of this build: the down-sampled directory must exist."""
    poses_arr = np.load(os.path.join(basedir, "poses_bounds.npy"))
    poses = poses_arr[:, :-2].reshape([-1, 3, 5]).transpose([1, 2, 0])
    bds = poses_arr[:, -2:].transpose([1, 0])
    from PIL import Image
    with Image.open(_list_images(os.path.join(basedir, "images"))[0]) as im:
        sh = (im.size[1], im.size[0])
    sfx = ""
    if factor is not None:
        sfx = f"_{factor}"
    elif height is not None:
        factor = sh[0] / float(height)
        width = int(sh[1] / factor)
        sfx = f"_{width}x{height}"
    elif width is not None:
        factor = sh[1] / float(width)
        height = int(sh[0] / factor)
        sfx = f"_{width}x{height}"
    else:
        factor = 1
    imgdir = os.path.join(basedir, "images" + sfx)
    if not os.path.exists(imgdir):
        raise FileNotFoundError(f"{imgdir} does not exist (create it by down-sampling `images/`; the reference "
                                f"shells out to ImageMagick mogrify for this)")
    imgfiles = _list_images(imgdir)
    if poses.shape[-1] != len(imgfiles):
        raise ValueError(f"Mismatch between imgs {len(imgfiles)} and poses {poses.shape[-1]}")
    with Image.open(imgfiles[0]) as im:
        sh = (im.size[1], im.size[0])
    poses[:2, 4, :] = np.array(sh[:2]).reshape([2, 1])
    poses[2, 4, :] = poses[2, 4, :] * 1.0 / factor
    return poses, bds, imgfiles


@DATASETS.register_module()
class LLFFDataset(Dataset):
    """Items are (pose [3,4] with the axis flip, focal [1], image [H,W,3], min_depth [1], max_depth [1])."""
    data_wrapper: Callable = LLFFDatasetWrapper

    def __init__(self, base_dir, split, test_skip=8, factor=8, recenter=True, bd_factor=0.75, spherify=False,
                 path_zflat=False, debug=False):
        if split not in ["train", "val", "test"]:
            raise ValueError(f"Invalid split: {split}.")
        poses, bds, imgfiles = load_llff_data(base_dir, factor=factor)
        # [down, right, back] -> [right, up, back]; N first (:51-53)
        poses = np.concatenate([poses[:, 1:2, :], -poses[:, 0:1, :], poses[:, 2:, :]], 1)
        poses = np.moveaxis(poses, -1, 0).astype(np.float32)
        bds = np.moveaxis(bds, -1, 0).astype(np.float32)
        sc = 1.0 if bd_factor is None else 1.0 / (bds.min() * bd_factor)  # (:56-58)
        poses[:, :3, 3] *= sc
        bds *= sc
        if recenter:
            poses = recenter_poses(poses)
        if spherify:
            poses, render_poses, bds = spherify_poses(poses, bds)
        else:
            c2w = poses_avg(poses)
            up = normalize(poses[:, :3, 1].sum(0))
            close_depth, inf_depth = bds.min() * 0.9, bds.max() * 5.0
            dt = 0.75
            focal = 1.0 / (((1.0 - dt) / close_depth + dt / inf_depth))
            zdelta = close_depth * 0.2
            rads = np.percentile(np.abs(poses[:, :3, 3]), 90, 0)
            c2w_path = c2w
            n_views, n_rots = 120, 2
            if path_zflat:
                zloc = -close_depth * 0.1
                c2w_path[:3, 3] = c2w_path[:3, 3] + zloc * c2w_path[:3, 2]
                rads[2] = 0.0
                n_rots = 1
                n_views //= 2  # the reference's `/= 2` makes a float count that np.linspace rejects
            render_poses = render_path_spiral(c2w_path, up, rads, focal, zdelta, zrate=0.5, rots=n_rots, N=n_views)
        self.render_poses = np.array(render_poses).astype(np.float32)
        c2w = poses_avg(poses)
        if test_skip > 0:
            i_test = np.arange(0, len(imgfiles), test_skip)
        else:
            i_test = np.array([np.argmin(np.sum(np.square(c2w[:3, 3] - poses[:, :3, 3]), -1))])
        poses = poses.astype(np.float32)
        imgfiles = np.array(imgfiles)
        if split in ("val", "test"):
            sel = i_test
        else:
            sel = np.array([i for i in range(len(imgfiles)) if i not in i_test])
        self.poses, self.imgfiles, self.bds = poses[sel], imgfiles[sel], bds[sel]
        calib = np.eye(4).astype(np.float32)
        calib[1, 1] = calib[2, 2] = -1.0
        self.calib_mat = calib

    def __getitem__(self, index: int) -> Tuple[torch.Tensor, ...]:
        pose = self.poses[index].astype(np.float32)
        focal = pose[2, -1]
        pose = pose[:, :4] @ self.calib_mat
        min_depth, max_depth = self.bds[index].astype(np.float32)
        img = load_image(self.imgfiles[index])
        return (torch.from_numpy(pose), torch.FloatTensor([focal]), torch.from_numpy(img),
                torch.FloatTensor([min_depth]), torch.FloatTensor([max_depth]))

    def __len__(self):
        return len(self.imgfiles)
