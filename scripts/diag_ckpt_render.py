"""tests/test_gpu_checkpoint.py::test_validation_render_matches_volume_render, taken apart: the trained
fixture, then validation_render and volume_render (the test's arguments) twice each, with gradients
enabled (the differentiable path: training forward kernel) and under no_grad (the render kernel), and
the maximum difference between every pair.  Diagnostic, not a test."""
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nerfmi  # noqa: E402,F401
from test_dataset import _config, write_synthetic_scene  # noqa: E402


def main():
    from nerfmi.dataset import NeRFDataset
    from nerfmi.render import volume_render
    from nerfmi.train import train_nerf, validation_render
    root = tempfile.mkdtemp()
    write_synthetic_scene(root, n=4, H=24, W=24, seed=2)
    cfg = _config(root, batch_size=256)
    np.random.seed(0)
    torch.manual_seed(0)
    ds = NeRFDataset(cfg)
    model = train_nerf(cfg, ds, save_dir=os.path.join(root, "ckpt"), num_iterations=4, checkpoint_every=2, seed=1,
                       log_every=0)
    val = ds.get_rays(idx=len(ds) - 1)
    print("near/far", ds.near, ds.far, "samples", cfg.num_samples, "importance", cfg.num_importance,
          "app idx", val["appearance_idx"], len(ds) - 1, "use_appearance", cfg.use_appearance)
    out = {}
    out["val_a"] = validation_render(model, ds, cfg, 7, root)
    out["val_b"] = validation_render(model, ds, cfg, 8, root)

    def vr(near, far, nimp):
        return volume_render(model, val["rays_o"][:1000], val["rays_d"][:1000], near, far, cfg.num_samples, nimp,
                             appearance_embedding=ds.appearance_embeddings[len(ds) - 1], perturb=False)[:2]
    out["test_a"] = vr(2.0, 6.0, 0)
    out["test_b"] = vr(2.0, 6.0, 0)
    out["test_dsnear"] = vr(ds.near, ds.far, cfg.num_importance)
    with torch.no_grad():
        out["nograd"] = vr(2.0, 6.0, 0)
    keys = list(out)
    for i, a in enumerate(keys):
        for b in keys[i + 1:]:
            dr = (out[a][0] - out[b][0]).abs().max().item()
            dd = (out[a][1].reshape(-1) - out[b][1].reshape(-1)).abs().max().item()
            print(f"{a:12s} vs {b:12s}: max |d rgb| {dr:.3e}  max |d depth| {dd:.3e}")


if __name__ == "__main__":
    main()
