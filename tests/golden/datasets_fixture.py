"""Write the synthetic datasets stored in tests/golden/datasets.npz back to disk in the reference's formats
(shared by make_golden_datasets.py and the loader tests)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
from PIL import Image


def write_blender(root: Path, blender_json: dict, train_png: np.ndarray, test_png: np.ndarray):
    root = Path(root)
    for split, pngs in (("train", train_png), ("test", test_png)):
        meta = json.loads(str(blender_json[split]))
        (root / split).mkdir(parents=True, exist_ok=True)
        (root / f"transforms_{split}.json").write_text(json.dumps(meta))
        for f, px in zip(meta["frames"], pngs):
            Image.fromarray(px, "RGBA").save(root / f"{f['file_path']}.png")


def write_llff(root: Path, poses_bounds: np.ndarray, full_png: np.ndarray, small_png: np.ndarray):
    root = Path(root)
    (root / "images").mkdir(parents=True, exist_ok=True)
    (root / "images_8").mkdir(parents=True, exist_ok=True)
    np.save(root / "poses_bounds.npy", poses_bounds)
    Image.fromarray(full_png[0], "RGB").save(root / "images" / "IMG_0000.png")
    for i, px in enumerate(small_png):
        Image.fromarray(px, "RGB").save(root / "images_8" / f"image{i:03d}.png")
