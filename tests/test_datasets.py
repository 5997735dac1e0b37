"""Data loaders against the reference's own loaders (golden: tests/golden/make_golden_datasets.py), on CPU."""
import numpy as np
import pytest
import torch

from datasets_fixture import write_blender, write_llff


@pytest.fixture(scope="module")
def ds_golden(golden):
    return golden("datasets")


@pytest.fixture(scope="module")
def dirs(ds_golden, tmp_path_factory):
    root = tmp_path_factory.mktemp("data")
    g = ds_golden
    write_blender(root / "lego", {"train": g["blender_train_json"], "test": g["blender_test_json"]},
                  g["blender_train_png"], g["blender_test_png"])
    write_llff(root / "fern", g["llff_poses_bounds"], g["llff_full_png"], g["llff_small_png"])
    return root


@pytest.mark.parametrize("split", ["train", "test"])
def test_blender_matches_reference(dirs, ds_golden, split):
    from yanerf_amd.datasets import DATASETS
    ds = DATASETS.build(dict(type="BlenderDataset", base_dir=str(dirs / "lego"), split=split, scale_down=1,
                             test_skip=8))
    g = ds_golden
    assert len(ds) == len(g[f"blender_{split}_pose"])
    assert [ds.H, ds.W] == list(g[f"blender_{split}_HW"])
    for i in range(len(ds)):
        pose, focal, img = ds[i]
        np.testing.assert_array_equal(pose.numpy(), g[f"blender_{split}_pose"][i])
        np.testing.assert_array_equal(focal.numpy(), g[f"blender_{split}_focal"][i])
        np.testing.assert_array_equal(img.numpy(), g[f"blender_{split}_img"][i])  # alpha dropped, /255


def test_blender_errors_and_scale_down(dirs):
    from yanerf_amd.datasets import BlenderDataset
    with pytest.raises(ValueError):
        BlenderDataset(str(dirs / "lego"), "bad")
    ds = BlenderDataset(str(dirs / "lego"), "train", scale_down=2)
    pose, focal, img = ds[0]
    assert (ds.H, ds.W) == (4, 4) and img.shape == (4, 4, 3)  # parity with cv2 itself unpinned (no cv2 here)
    full = BlenderDataset(str(dirs / "lego"), "train")
    assert abs(float(focal) - float(full[0][1]) / 2) < 1e-6


@pytest.mark.parametrize("tag,kw", [("spiral", dict(recenter=True, spherify=False)),
                                    ("sphere", dict(recenter=True, spherify=True)),
                                    ("norecenter", dict(recenter=False, spherify=False, bd_factor=None))])
@pytest.mark.parametrize("split", ["train", "test"])
def test_llff_matches_reference(dirs, ds_golden, tag, kw, split):
    from yanerf_amd.datasets import DATASETS
    ds = DATASETS.build(dict(type="LLFFDataset", base_dir=str(dirs / "fern"), split=split, test_skip=4, factor=8, **kw))
    p = f"llff_{tag}_{split}"
    g = ds_golden
    np.testing.assert_allclose(ds.poses, g[f"{p}_poses"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(ds.bds, g[f"{p}_bds"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(ds.render_poses, g[f"{p}_render_poses"], rtol=0, atol=1e-5)
    import os
    assert [os.path.basename(f) for f in ds.imgfiles] == list(g[f"{p}_files"])
    for i in range(len(ds)):
        pose, focal, img, near, far = ds[i]
        np.testing.assert_allclose(pose.numpy(), g[f"{p}_item_pose"][i], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(focal.numpy(), g[f"{p}_item_focal"][i])
        np.testing.assert_array_equal(img.numpy(), g[f"{p}_item_img"][i])
        np.testing.assert_allclose(near.numpy(), g[f"{p}_item_near"][i], rtol=0, atol=1e-6)
        np.testing.assert_allclose(far.numpy(), g[f"{p}_item_far"][i], rtol=0, atol=1e-6)


def test_llff_missing_downsampled_dir(tmp_path, ds_golden):
    from yanerf_amd.datasets import LLFFDataset
    g = ds_golden
    write_llff(tmp_path, g["llff_poses_bounds"], g["llff_full_png"], g["llff_small_png"])
    with pytest.raises(FileNotFoundError):
        LLFFDataset(str(tmp_path), "train", factor=4)


def test_device_image_set_and_sampler_order(dirs):
    from torch.utils.data import DistributedSampler

    from yanerf_amd.datasets import BlenderDataset, DeviceImageSet, LLFFDataset
    ds = BlenderDataset(str(dirs / "lego"), "test", test_skip=1)  # 16 frames
    dev = DeviceImageSet(ds, "cpu")
    assert len(dev) == 16 and dev.images.shape == (16, 8, 8, 3) and dev.near is None
    pose, focal, img, near, far = dev.item(3)
    np.testing.assert_array_equal(pose[0].numpy(), ds[3][0][:3, :4].numpy())
    np.testing.assert_array_equal(img[0].numpy(), ds[3][2].numpy())
    for world in (1, 2, 3):
        for rank in range(world):
            for epoch in (0, 5):
                ref = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=7, drop_last=True)
                ref.set_epoch(epoch)
                assert list(dev.epoch_order(epoch, rank, world, shuffle=True, seed=7, drop_last=True)) == list(ref)
                ref = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=False, drop_last=False)
                assert list(dev.epoch_order(epoch, rank, world, shuffle=False, drop_last=False)) == list(ref)
    ll = DeviceImageSet(LLFFDataset(str(dirs / "fern"), "train", test_skip=4, factor=8), "cpu")
    assert ll.near is not None and ll.near.shape == (len(ll),) and torch.all(ll.far > ll.near)


@pytest.mark.parametrize("name,sub,splits", [("lego", "lego", ("train", "test")), ("fern", "fern", ("train", "test"))])
def test_product_config_datasets_build(dirs, name, sub, splits):
    """The `datasets:` entries of the product configs (lego.yml / fern.yml) build through DATASETS as in run.py:95-110
    (base_dir pointed at the synthetic fixture; fern.yml's defaults factor=8 / test_skip=8 apply)."""
    import copy

    import yanerf_boot
    from yanerf_amd.datasets import DATASETS
    from yanerf_amd.utils.config import Config
    cfg = Config.fromfile(str(yanerf_boot.PKG_DIR / f"configs/nerf/{name}.yml"))
    for entry in cfg.datasets:
        if entry["split"] not in splits:
            continue
        e = copy.deepcopy(dict(entry))
        e["base_dir"] = str(dirs / sub)
        ds = DATASETS.build(e)
        assert len(ds) > 0
        item = ds[0]
        assert item[0].shape[-1] == 4 and item[2].shape[-1] == 3
