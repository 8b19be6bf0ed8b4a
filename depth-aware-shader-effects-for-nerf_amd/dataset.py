"""Ray batches for training (src/dataset.py:9-277 of the reference), without torchvision.

``NeRFDataset`` reads a nerf_synthetic scene (transforms_<split>.json + RGBA PNGs) when it is
present under config.dataset_path, exactly as dataset.py:29-83,125-209 do: focal from
camera_angle_x, images as float RGB in [0,1] (ToTensor), one appearance embedding per image
(randn(n_images, 32)).  ``get_rays(idx=None, batch_size=None)`` returns the same dict as
dataset.py:211-277: a whole image for ``idx``, otherwise ``batch_size`` distinct random pixels
of one random image (np.random.randint / np.random.choice(replace=False), dataset.py:249-260).

``SyntheticNeRFDataset`` is the stand-in used when no dataset exists (none does in this
environment): the same interface over ``n_images`` poses on the nerf_synthetic camera sphere
(radius 4.0311, looking at the origin), whose pixel colours are rendered on the fly by a fixed
random-init "teacher" NeRF through nerfmi's own renderer (coarse, perturb=False).  Training a
student on it is a well-posed regression, so losses fall as they would on real images.
Ray generation runs in the HIP get_rays kernel; pixels are selected on the host with numpy's
global generator as the reference does.
"""
import json
import os

import numpy as np
import torch

from . import _lib, cameras
from .ray_utils import get_rays as _get_rays

SYNTHETIC_RADIUS = 4.031128857175383     # |t| of the Blender nerf_synthetic train poses


class _RayBatches:
    """get_rays(idx=None, batch_size=None) of dataset.py:206-277 over self.c2w / self._pixels."""

    def __len__(self):
        return len(self.c2w)

    def _rays(self, idx):
        o, d = _get_rays(self.H, self.W, self.focal, self.c2w[idx].to(_lib.device()))
        return o.reshape(-1, 3), d.reshape(-1, 3)

    def _app_idx(self, idx):
        return idx if self.use_appearance else -1                                   # dataset.py:167-170

    def get_rays(self, idx=None, batch_size=None):
        if batch_size is None:
            batch_size = self.config.batch_size
        if idx is not None:
            o, d = self._rays(idx)
            rgb, alpha = self._pixels(idx, None, o, d)
            return {"rays_o": o, "rays_d": d, "rgb": rgb, "alpha": alpha,
                    "appearance_idx": self._app_idx(idx), "img_idx": idx}
        img_idx = np.random.randint(0, len(self))                                   # dataset.py:250
        o, d = self._rays(img_idx)
        sel = np.random.choice(self.H * self.W, size=batch_size, replace=False)    # dataset.py:260
        sel_t = torch.from_numpy(sel).to(o.device)
        o, d = o[sel_t].contiguous(), d[sel_t].contiguous()
        rgb, alpha = self._pixels(img_idx, sel, o, d)
        return {"rays_o": o, "rays_d": d, "rgb": rgb, "alpha": alpha,
                "appearance_idx": self._app_idx(img_idx), "img_idx": img_idx}

    def __getitem__(self, idx):
        """dataset.py:129-204: {'img' (3,H,W), 'alpha' (1,H,W) or None, 'c2w' (4,4),
        'appearance_idx', 'img_idx'} on the CPU."""
        if idx < 0:
            idx += len(self)
        if not 0 <= idx < len(self):
            raise IndexError(f"image index {idx} out of range for {len(self)} images")
        rgb, alpha = self._image_chw(idx)
        return {"img": rgb, "alpha": alpha, "c2w": self.c2w[idx].clone(), "appearance_idx": self._app_idx(idx),
                "img_idx": idx}


def _appearance_table(n, dim):
    """dataset.py:79-83: one trainable embedding per image, randn(n, dim) as an nn.Parameter."""
    return torch.nn.Parameter(torch.randn(n, dim))


class NeRFDataset(_RayBatches):
    """dataset.py:9-204: 'nerf_synthetic' scenes (transforms_<split>.json + RGBA PNGs under
    dataset_path/scene) and the custom format (dataset_path/../transforms.json, all frames but
    the last for 'train', the last one otherwise).  Decoded images are cached, where the
    reference decodes a PNG on every batch (dataset.py:156,250-251)."""

    def __init__(self, config, split="train"):
        from PIL import Image
        self.config, self.split = config, split
        self._cache = {}
        self.dataset_type = getattr(config, "dataset_type", "nerf_synthetic")
        if self.dataset_type == "nerf_synthetic":                                 # dataset.py:29-83
            scene_path = os.path.join(config.dataset_path, config.scene)
            with open(os.path.join(scene_path, f"transforms_{split}.json")) as f:
                self.meta = json.load(f)
            self.frames = self.meta["frames"]
            self.paths = []
            for fr in self.frames:
                p = fr["file_path"]
                p = p[2:] if p.startswith("./") else p
                self.paths.append(os.path.join(scene_path, p + ".png"))
            with Image.open(self.paths[0]) as img:
                self.W, self.H = img.size
            width = self.W
            self.near, self.far = config.near, config.far
        else:                                                                      # dataset.py:85-124
            with open(os.path.join(config.dataset_path, "../transforms.json")) as f:
                self.meta = json.load(f)
            self.frames = self.meta["frames"][:-1] if split == "train" else self.meta["frames"][-1:]
            self.paths = [os.path.join(config.dataset_path, fr["file_path"]) for fr in self.frames]
            self.H, self.W = self.meta["h"], self.meta["w"]
            width = self.meta["w"]
            self.near, self.far = 2.0, 6.0
        if "camera_angle_x" in self.meta:                                          # dataset.py:65-71
            self.focal = 0.5 * width / np.tan(0.5 * self.meta["camera_angle_x"])
        elif "fl_x" in self.meta:
            self.focal = self.meta["fl_x"]
        else:
            self.focal = width / (2 * np.tan(np.radians(55) / 2))
        self.use_appearance = config.use_appearance
        self.appearance_embeddings = _appearance_table(len(self.frames), config.appearance_dim) \
            if self.use_appearance else None
        self.c2w = [torch.tensor(fr["transform_matrix"], dtype=torch.float32) for fr in self.frames]

    def _image_chw(self, idx):
        """ToTensor of the image file (dataset.py:156-161): rgb (3,H,W) in [0,1], alpha (1,H,W)
        (ones without an alpha channel; None for the custom format, dataset.py:182,190).  The decoded
        file is cached as its uint8 HWC array (a quarter of the float tensor's size; the reference
        decodes on every access) and converted on every call, so callers get fresh tensors."""
        if idx not in self._cache:
            from PIL import Image
            with Image.open(self.paths[idx]) as img:
                if self.dataset_type != "nerf_synthetic":
                    img = img.convert("RGB")
                arr = np.asarray(img, dtype=np.uint8)
            if arr.ndim == 2:
                arr = arr[..., None]
            self._cache[idx] = np.ascontiguousarray(arr)
        arr = self._cache[idx]
        t = torch.from_numpy(arr).permute(2, 0, 1).float().div(255)              # ToTensor
        rgb = t[:3]
        if self.dataset_type != "nerf_synthetic":
            alpha = None
        else:
            alpha = t[3:4] if t.shape[0] == 4 else torch.ones_like(t[:1])
        return rgb, alpha

    def _pixels(self, idx, sel, o, d):
        rgb, alpha = self._image_chw(idx)
        rgb = rgb.permute(1, 2, 0).reshape(-1, 3)                                   # dataset.py:235,265
        alpha = alpha.permute(1, 2, 0).reshape(-1, 1) if alpha is not None else None
        if sel is not None:
            rgb = rgb[sel]
            alpha = alpha[sel] if alpha is not None else None
        dev = o.device
        return rgb.to(dev), (alpha.to(dev) if alpha is not None else None)


class SyntheticNeRFDataset(_RayBatches):
    """Teacher-rendered stand-in for a nerf_synthetic training split (module docstring)."""

    def __init__(self, config, n_images=100, H=800, W=800, teacher_seed=1234, pose_seed=0, n_samples=None):
        from .models import NeRF
        self.config = config
        self.H, self.W = H, W
        self.focal = cameras.synthetic_focal(W)
        self.near, self.far = config.near, config.far
        self.use_appearance = config.use_appearance
        rng = np.random.default_rng(pose_seed)
        self.c2w = []
        for _ in range(n_images):             # upper hemisphere, as the Blender train views
            theta = rng.uniform(0, 2 * np.pi)
            elev = rng.uniform(np.radians(5), np.radians(85))
            pos = SYNTHETIC_RADIUS * np.array([np.cos(elev) * np.sin(theta), np.sin(elev),
                                               np.cos(elev) * np.cos(theta)])
            self.c2w.append(torch.tensor(cameras.look_at_c2w(pos, np.zeros(3), np.array([0, 1, 0])),
                                         dtype=torch.float32))
        g = torch.Generator().manual_seed(teacher_seed)
        fork = torch.random.fork_rng(devices=[])
        with fork:
            torch.manual_seed(teacher_seed)
            self.teacher = NeRF(config).to(_lib.device()).eval()
            self.teacher_app = torch.randn(n_images, config.appearance_dim, generator=g)
        self.appearance_embeddings = _appearance_table(n_images, config.appearance_dim) \
            if self.use_appearance else None
        self.n_samples = n_samples or config.num_samples

    @torch.no_grad()
    def _pixels(self, idx, sel, o, d):
        from .render import volume_render
        app = self.teacher_app[idx].to(o.device) if self.use_appearance else None
        rgb, _, _ = volume_render(self.teacher, o, d, self.near, self.far, self.n_samples, 0,
                                  appearance_embedding=app, perturb=False)
        return rgb, torch.ones(rgb.shape[0], 1, device=o.device)

    def _image_chw(self, idx):
        o, d = self._rays(idx)
        rgb, alpha = self._pixels(idx, None, o, d)
        return (rgb.reshape(self.H, self.W, 3).permute(2, 0, 1).cpu().contiguous(),
                alpha.reshape(self.H, self.W, 1).permute(2, 0, 1).cpu().contiguous())


def make_dataset(config, split="train", **synthetic_kw):
    """NeRFDataset when the scene is on disk, else SyntheticNeRFDataset."""
    path = os.path.join(config.dataset_path, config.scene, f"transforms_{split}.json")
    if os.path.exists(path):
        return NeRFDataset(config, split)
    return SyntheticNeRFDataset(config, **synthetic_kw)
