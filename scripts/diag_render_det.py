"""Repeat the render MLP (nerf_mlp_forward: mlp16s_kernel under f16x3) on identical inputs, with other
kernels in between (a training forward, which leaves other data in LDS; or nothing), and report every
repetition that differs from the first: which samples (position in their 32-sample wave block) and
outputs.  Shapes: R rays x N samples for several (R, N).  NERFMI_LIB selects the library.  Diagnostic."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import nerfmi  # noqa: E402
from nerfmi import _lib as L  # noqa: E402
from nerfmi.ray_utils import linspace_table  # noqa: E402
from nerfmi.train import Trainer  # noqa: E402

REPS = int(os.environ.get("REPS", "12"))


def main():
    lib, P, s = L.load(), L.ptr, L.stream()
    dev = L.device()
    torch.manual_seed(0)
    tr = Trainer(nerfmi.Config())
    L.check(lib.nerf_pack_weights(tr.param_ptrs, P(tr.packed), s), "pack")   # (a Trainer packs in its step)
    g = torch.Generator().manual_seed(1)
    app = torch.randn(1, 32, generator=g).to(dev)
    for R, N in ((576, 32), (576, 64), (1000, 32), (4096, 64), (777, 48)):
        M = R * N
        o = (torch.randn(R, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
        d = torch.randn(R, 3, generator=g).to(dev)
        d[:, 2] = -d[:, 2].abs() - 1.0
        t_rand = torch.rand(R, N, generator=g).to(dev)
        dn, z = torch.empty(R, 3, device=dev), torch.empty(R, N, device=dev)
        feat, encd = torch.empty(R, 256, device=dev), torch.empty(R, 32, device=dev)
        L.check(lib.nerf_normalize_dirs(P(d), R, P(dn), s), "normalize")
        L.check(lib.nerf_sample_stratified(P(o), P(dn), R, tr.near, tr.far, N, P(linspace_table(N, dev)), 1,
                                           P(t_rand), 0, P(z), None, s), "stratified")
        L.check(lib.nerf_ray_features_train(P(tr.packed), P(dn), R, P(app), 1, P(feat), P(encd), s), "features")
        # an LDS scribbler: the training forward on the same rays (other LDS layout and contents)
        save = torch.empty(L.tile_rows(M), L.SAVE_ROW, device=dev)
        masks = torch.empty(M, L.MASK_ROW, dtype=torch.int32, device=dev)
        rgb_t, sig_t = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)

        def render(mode):
            if mode == "scribble":
                L.check(lib.nerf_mlp_forward_train(P(tr.packed), P(o), P(dn), P(z), R, N, P(feat), P(encd), P(rgb_t),
                                                   P(sig_t), P(save), P(masks), s), "train forward")
            rgb, sigma = torch.full((M, 3), float("nan"), device=dev), torch.full((M,), float("nan"), device=dev)
            L.check(lib.nerf_mlp_forward(P(tr.packed), P(o), P(dn), P(z), R, N, P(feat), P(rgb), P(sigma), None, 0, s),
                    "render forward")
            torch.cuda.synchronize()
            return rgb.cpu(), sigma.cpu()

        for mode in ("plain", "scribble"):
            ref = render(mode)
            bad = 0
            for rep in range(REPS):
                cur = render("scribble" if rep % 2 else "plain")
                ne = (ref[0] != cur[0]).any(1) | (ref[1] != cur[1])
                ne |= torch.isnan(cur[0]).any(1) | torch.isnan(cur[1])
                if ne.any():
                    bad += 1
                    rows = ne.nonzero().flatten().numpy()
                    if bad <= 2:
                        print(f"  R={R} N={N} ref {mode} rep {rep}: {len(rows)} samples differ in "
                              f"{len(np.unique(rows // 32))} waves; first {rows[:8].tolist()}; lane histogram "
                              f"{np.bincount(rows % 32, minlength=32).tolist()}")
            print(f"R={R} N={N} reference after '{mode}': {bad} of {REPS} repetitions differ")
    print(f"library: {os.environ.get('NERFMI_LIB') or 'in-tree'}, arith {L.get_mlp_arith()}")


if __name__ == "__main__":
    main()
