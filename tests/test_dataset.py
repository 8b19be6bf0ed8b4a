"""NeRFDataset (src/dataset.py:9-277 of the reference) on a synthetic nerf_synthetic tree and a
synthetic custom-format tree, written by the tests (no dataset exists here).

Host tests: transforms parsing, focal, ToTensor semantics of __getitem__, the appearance table as
an nn.Parameter.  GPU tests: get_rays (whole image and random batch) against the oracle's
get_rays and the PNG pixels."""
import json
import os

import numpy as np
import pytest
import torch

import nerfmi
from nerfmi.dataset import NeRFDataset

CAMERA_ANGLE_X = 0.6911112070083618


def _pose(k):
    th = 0.7 * k
    c, s = np.cos(th), np.sin(th)
    return [[c, 0.0, s, 4.0 * s], [0.0, 1.0, 0.0, 0.3 * k], [-s, 0.0, c, 4.0 * c], [0.0, 0.0, 0.0, 1.0]]


def write_synthetic_scene(root, scene="lego", split="train", n=3, H=12, W=16, seed=0, mode="RGBA"):
    """A nerf_synthetic-style tree: <root>/<scene>/transforms_<split>.json + ./<split>/r_<k>.png."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    sdir = os.path.join(root, scene)
    os.makedirs(os.path.join(sdir, split), exist_ok=True)
    frames, pix = [], []
    for k in range(n):
        ch = 4 if mode == "RGBA" else 3
        arr = rng.integers(0, 256, size=(H, W, ch), dtype=np.uint8)
        Image.fromarray(arr, mode).save(os.path.join(sdir, split, f"r_{k}.png"))
        frames.append({"file_path": f"./{split}/r_{k}", "rotation": 0.0, "transform_matrix": _pose(k)})
        pix.append(arr)
    with open(os.path.join(sdir, f"transforms_{split}.json"), "w") as f:
        json.dump({"camera_angle_x": CAMERA_ANGLE_X, "frames": frames}, f)
    return pix


def _config(root, scene="lego", use_appearance=True, batch_size=64):
    cfg = nerfmi.Config()
    cfg.dataset_path = str(root)
    cfg.scene = scene
    cfg.use_appearance = use_appearance
    cfg.batch_size = batch_size
    return cfg


def test_synthetic_scene_metadata_and_getitem(tmp_path):
    pix = write_synthetic_scene(tmp_path, n=3, H=12, W=16)
    torch.manual_seed(5)
    ds = NeRFDataset(_config(tmp_path))
    assert len(ds) == 3 and (ds.H, ds.W) == (12, 16)
    assert ds.focal == 0.5 * 16 / np.tan(0.5 * CAMERA_ANGLE_X)                   # dataset.py:66
    assert (ds.near, ds.far) == (2.0, 6.0)
    assert isinstance(ds.appearance_embeddings, torch.nn.Parameter)                # dataset.py:81-83
    torch.manual_seed(5)
    assert torch.equal(ds.appearance_embeddings.data, torch.randn(3, 32))
    for k in (0, 2, -1):
        s = ds[k]
        kk = k % 3
        assert set(s) == {"img", "alpha", "c2w", "appearance_idx", "img_idx"}
        assert s["img"].shape == (3, 12, 16) and s["alpha"].shape == (1, 12, 16)
        # ToTensor: uint8 -> float32 / 255, CHW
        want = torch.from_numpy(pix[kk]).permute(2, 0, 1).float().div(255)
        assert torch.equal(s["img"], want[:3]) and torch.equal(s["alpha"], want[3:4])
        assert torch.equal(s["c2w"], torch.tensor(_pose(kk), dtype=torch.float32))
        assert s["appearance_idx"] == kk and s["img_idx"] == kk
    with pytest.raises(IndexError):
        ds[3]


def test_rgb_images_get_unit_alpha_and_no_appearance(tmp_path):
    write_synthetic_scene(tmp_path, n=2, mode="RGB")
    ds = NeRFDataset(_config(tmp_path, use_appearance=False))
    s = ds[1]
    assert torch.equal(s["alpha"], torch.ones(1, 12, 16))                        # dataset.py:161
    assert s["appearance_idx"] == -1                                               # dataset.py:170
    assert ds.appearance_embeddings is None


def test_custom_format(tmp_path):
    """dataset.py:85-124: <dataset_path>/../transforms.json; all frames but the last for 'train'."""
    from PIL import Image
    data = tmp_path / "custom" / "images"
    data.mkdir(parents=True)
    rng = np.random.default_rng(1)
    frames = []
    for k in range(4):
        Image.fromarray(rng.integers(0, 256, (10, 8, 4), dtype=np.uint8), "RGBA").save(data / f"f{k}.png")
        frames.append({"file_path": f"f{k}.png", "transform_matrix": _pose(k)})
    with open(tmp_path / "custom" / "transforms.json", "w") as f:
        json.dump({"fl_x": 9.5, "w": 8, "h": 10, "frames": frames}, f)
    cfg = _config(tmp_path)
    cfg.dataset_type = "custom"
    cfg.dataset_path = str(data)
    tr = NeRFDataset(cfg, "train")
    va = NeRFDataset(cfg, "val")
    assert len(tr) == 3 and len(va) == 1
    assert (tr.H, tr.W, tr.focal) == (10, 8, 9.5)
    s = va[0]
    assert s["img"].shape == (3, 10, 8) and s["alpha"] is None                     # convert('RGB')
    assert torch.equal(s["c2w"], torch.tensor(_pose(3), dtype=torch.float32))


def test_make_dataset_prefers_files_on_disk(tmp_path):
    from nerfmi.dataset import make_dataset
    write_synthetic_scene(tmp_path, n=2)
    assert isinstance(make_dataset(_config(tmp_path)), NeRFDataset)


@pytest.mark.gpu
def test_get_rays_whole_image_and_batches(tmp_path):
    from oracle import nerf_oracle as O
    pix = write_synthetic_scene(tmp_path, n=3, H=12, W=16)
    ds = NeRFDataset(_config(tmp_path, batch_size=40))
    full = ds.get_rays(idx=1)
    o_ref, d_ref = O.get_rays(12, 16, ds.focal, torch.tensor(_pose(1), dtype=torch.float32))
    assert torch.equal(full["rays_o"].cpu(), o_ref.reshape(-1, 3))
    assert torch.equal(full["rays_d"].cpu(), d_ref.reshape(-1, 3))
    px = torch.from_numpy(pix[1]).float().div(255).reshape(-1, 4)
    assert torch.equal(full["rgb"].cpu(), px[:, :3]) and torch.equal(full["alpha"].cpu(), px[:, 3:])
    assert full["appearance_idx"] == 1 and full["img_idx"] == 1
    # random batch: np.random.randint image, np.random.choice(replace=False) pixels (dataset.py:250,260)
    np.random.seed(3)
    b = ds.get_rays()
    np.random.seed(3)
    k = np.random.randint(0, 3)
    sel = np.random.choice(12 * 16, size=40, replace=False)
    assert b["img_idx"] == k and b["rays_o"].shape == (40, 3)
    o_ref, d_ref = O.get_rays(12, 16, ds.focal, torch.tensor(_pose(k), dtype=torch.float32))
    assert torch.equal(b["rays_d"].cpu(), d_ref.reshape(-1, 3)[sel])
    px = torch.from_numpy(pix[k]).float().div(255).reshape(-1, 4)
    assert torch.equal(b["rgb"].cpu(), px[sel, :3])
    assert ds.get_rays(batch_size=7)["rays_o"].shape == (7, 3)
