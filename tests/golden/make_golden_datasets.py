"""Golden vectors for the data loaders, made by running the REFERENCE loaders on tiny synthetic datasets.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden_datasets.py

It writes small synthetic datasets in the reference's on-disk formats (a nerf_synthetic `transforms_*.json` + RGBA
PNGs; an LLFF `poses_bounds.npy` + `images/` + `images_8/` PNGs) into a temp dir, loads them with
yanerf.dataset.{BlenderDataset, LLFFDataset} from /root/reference (third-party stand-ins from tests/golden/_stubs:
imageio is PIL-backed, cv2 is import-only, so only scale_down == 1 is exercised), and stores the dataset FILES' data
(JSON text, pixel arrays, poses_bounds) as inputs and the reference's items / pose products as expected outputs in
tests/golden/datasets.npz. The tests rebuild the same files from the fixture and compare our loaders.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("YANERF_REFERENCE", "/root/reference"))
sys.path.insert(0, str(HERE / "_stubs"))
sys.path.insert(0, str(REF))
sys.path.insert(0, str(HERE))

import torch  # noqa: E402

_six = types.ModuleType("torch._six")
_six.string_classes = (str, bytes)
sys.modules.setdefault("torch._six", _six)

from datasets_fixture import write_blender, write_llff  # noqa: E402


def rand_rot(rng):
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return q * np.sign(np.linalg.det(q))


def make_inputs(rng):
    # Blender: 4 train frames, 16 test frames (test_skip 8 -> 2), 8x8 RGBA
    def frames(n, prefix):
        out = []
        for i in range(n):
            m = np.eye(4)
            m[:3, :3] = rand_rot(rng)
            m[:3, 3] = rng.standard_normal(3) * 4.0
            out.append({"file_path": f"./{prefix}/r_{i}", "rotation": 0.012566, "transform_matrix": m.tolist()})
        return out
    blender = {
        "train": json.dumps({"camera_angle_x": 0.6911112070083618, "frames": frames(4, "train")}),
        "test": json.dumps({"camera_angle_x": 0.6911112070083618, "frames": frames(16, "test")}),
    }
    bl_train = (rng.random((4, 8, 8, 4)) * 255).astype(np.uint8)
    bl_test = (rng.random((16, 8, 8, 4)) * 255).astype(np.uint8)
    # LLFF: 10 views, images/ at 96x128, images_8/ at 12x16; poses of a forward-facing rig
    n = 10
    pb = np.zeros((n, 17))
    for i in range(n):
        R = rand_rot(rng) * 0.05 + np.array([[0, 1, 0], [1, 0, 0], [0, 0, -1.0]])
        R, _ = np.linalg.qr(R)
        t = rng.standard_normal(3) * 0.3
        hwf = np.array([96.0, 128.0, 110.0 + rng.random()])
        pb[i, :15] = np.concatenate([R, t[:, None], hwf[:, None]], 1).reshape(-1)
        pb[i, 15:] = [1.5 + rng.random(), 20.0 + 10 * rng.random()]
    ll_full = (rng.random((1, 96, 128, 3)) * 255).astype(np.uint8)
    ll_small = (rng.random((n, 12, 16, 3)) * 255).astype(np.uint8)
    return blender, bl_train, bl_test, pb, ll_full, ll_small


def main():
    from yanerf.dataset.blender_dataset import BlenderDataset
    from yanerf.dataset.llff_dataset import LLFFDataset
    rng = np.random.default_rng(123)
    blender, bl_train, bl_test, pb, ll_full, ll_small = make_inputs(rng)
    out = dict(blender_train_json=np.array(blender["train"]), blender_test_json=np.array(blender["test"]),
               blender_train_png=bl_train, blender_test_png=bl_test, llff_poses_bounds=pb, llff_full_png=ll_full,
               llff_small_png=ll_small)
    with tempfile.TemporaryDirectory() as tmp:
        bdir, ldir = Path(tmp) / "lego", Path(tmp) / "fern"
        write_blender(bdir, blender, bl_train, bl_test)
        write_llff(ldir, pb, ll_full, ll_small)
        for split in ("train", "test"):
            ds = BlenderDataset(str(bdir), split, scale_down=1, test_skip=8)
            items = [ds[i] for i in range(len(ds))]
            out[f"blender_{split}_pose"] = np.stack([it[0].numpy() for it in items])
            out[f"blender_{split}_focal"] = np.stack([it[1].numpy() for it in items])
            out[f"blender_{split}_img"] = np.stack([it[2].numpy() for it in items])
            out[f"blender_{split}_HW"] = np.array([ds.H, ds.W])
        for tag, kw in (("spiral", dict(recenter=True, spherify=False)), ("sphere", dict(recenter=True, spherify=True)),
                        ("norecenter", dict(recenter=False, spherify=False, bd_factor=None))):
            for split in ("train", "test"):
                ds = LLFFDataset(str(ldir), split, test_skip=4, factor=8, **kw)
                items = [ds[i] for i in range(len(ds))]
                p = f"llff_{tag}_{split}"
                out[f"{p}_poses"] = ds.poses.astype(np.float32)
                out[f"{p}_bds"] = ds.bds.astype(np.float32)
                out[f"{p}_render_poses"] = ds.render_poses.astype(np.float32)
                out[f"{p}_files"] = np.array([os.path.basename(f) for f in ds.imgfiles])
                out[f"{p}_item_pose"] = np.stack([it[0].numpy() for it in items])
                out[f"{p}_item_focal"] = np.stack([it[1].numpy() for it in items])
                out[f"{p}_item_img"] = np.stack([it[2].numpy() for it in items])
                out[f"{p}_item_near"] = np.stack([it[3].numpy() for it in items])
                out[f"{p}_item_far"] = np.stack([it[4].numpy() for it in items])
    np.savez_compressed(HERE / "datasets.npz", **out)
    print("wrote", HERE / "datasets.npz", sum(v.nbytes for v in out.values()), "bytes")


if __name__ == "__main__":
    main()
