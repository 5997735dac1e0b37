"""A dataset split resident in HBM.

The reference moves one image per step host-to-device through a DataLoader (runners/apis.py:55-57). Here the whole
split is uploaded once (Lego train: 100 x 800 x 800 x 3 fp32 = 768 MB, a small fraction of a 288 GB MI355X) and a
step indexes it on the device, so the timed training loop issues no H2D copy. The per-epoch order follows the
reference's samplers: DistributedSampler(shuffle=True) for training, a rank-strided split for evaluation
(runners/utils.py:112-131), with drop_last for training."""
from __future__ import annotations

from typing import Iterator, List, Optional

import numpy as np
import torch


class DeviceImageSet:
    def __init__(self, dataset, device, dtype=torch.float32, indices: Optional[List[int]] = None):
        idx = list(range(len(dataset))) if indices is None else list(indices)
        poses, focals, images, near, far = [], [], [], [], []
        for i in idx:
            item = dataset[i]
            poses.append(item[0][:3, :4])
            focals.append(item[1].reshape(-1)[:1])
            images.append(item[2])
            if len(item) >= 5:  # LLFF: per-image bounds
                near.append(item[3].reshape(-1)[:1])
                far.append(item[4].reshape(-1)[:1])
        self.device = torch.device(device)
        self.poses = torch.stack(poses).to(self.device, torch.float32).contiguous()    # [N,3,4]
        self.focals = torch.cat(focals).to(self.device, torch.float32).contiguous()    # [N]
        self.images = torch.stack(images).to(self.device, dtype).contiguous()           # [N,H,W,3]
        self.near = torch.cat(near).to(self.device).contiguous() if near else None      # [N] or None
        self.far = torch.cat(far).to(self.device).contiguous() if far else None
        self.H, self.W = int(self.images.shape[1]), int(self.images.shape[2])

    def __len__(self):
        return int(self.poses.shape[0])

    def item(self, i: int):
        """(pose [1,3,4], focal [1], image [1,H,W,3], near, far) as device views (no copies)."""
        near = None if self.near is None else self.near[i:i + 1]
        far = None if self.far is None else self.far[i:i + 1]
        return self.poses[i:i + 1], self.focals[i:i + 1], self.images[i:i + 1], near, far

    def epoch_order(self, epoch: int, rank: int = 0, world: int = 1, shuffle: bool = True, seed: int = 0,
                    drop_last: bool = True) -> Iterator[int]:
        """DistributedSampler order: a permutation seeded by seed + epoch (shuffle) padded / truncated to a multiple of
        the world size, then every world-th index starting at rank."""
        n = len(self)
        if shuffle:
            g = torch.Generator().manual_seed(seed + epoch)
            order = torch.randperm(n, generator=g).tolist()
        else:
            order = list(range(n))
        if drop_last and n % world:
            total = (n // world) * world
            order = order[:total]
        else:
            total = -(-n // world) * world
            order = order + order[: total - n]
        return iter(order[rank:total:world])
