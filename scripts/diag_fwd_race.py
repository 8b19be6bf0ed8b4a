"""Repeat the training forward (nerf_mlp_forward_train, production batch 4,096 rays x 64 samples) on
identical inputs and report where any repetition differs from the first.  MODE: "plain" (back to
back), "scribble" (a render forward on other inputs runs between, leaving other data in LDS), "side"
(a GEMM on a second stream runs concurrently).  Reported: rgb, sigma, save-row features
(by segment: h0..h7, enc_x, enc_d, r_dir, hd) and mask words, with the differing samples' positions in
their 32-sample wave block.  NERFMI_LIB selects the library.  Diagnostic for a race, not a test."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import nerfmi  # noqa: E402
from nerfmi import _lib as L  # noqa: E402
from nerfmi.ray_utils import linspace_table  # noqa: E402
from nerfmi.train import Trainer  # noqa: E402

REPS = int(os.environ.get("REPS", "30"))
SEGS = [("h%d" % j, o, o + 256) for j, o in enumerate([0, 256, 512, 768, 1088, 1344, 1600, 1856])] + \
       [("enc_x", 1024, 1088), ("enc_d", 2112, 2144), ("r_dir", 2144, 2272), ("hd", 2272, 2400)]


def main():
    lib, P, s = L.load(), L.ptr, L.stream()
    dev = L.device()
    cfg = nerfmi.Config()
    torch.manual_seed(0)
    tr = Trainer(cfg)
    L.check(lib.nerf_pack_weights(tr.param_ptrs, P(tr.packed), s), "pack")   # (a Trainer packs in its step)
    B, N = 4096, cfg.num_samples
    M = B * N
    g = torch.Generator().manual_seed(1)
    o = (torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
    d = torch.randn(B, 3, generator=g).to(dev)
    d[:, 2] = -d[:, 2].abs() - 1.0
    t_rand = torch.rand(B, N, generator=g).to(dev)
    dn, z = torch.empty(B, 3, device=dev), torch.empty(B, N, device=dev)
    feat, encd = torch.empty(B, 256, device=dev), torch.empty(B, 32, device=dev)
    L.check(lib.nerf_normalize_dirs(P(d), B, P(dn), s), "normalize")
    L.check(lib.nerf_sample_stratified(P(o), P(dn), B, tr.near, tr.far, N, P(linspace_table(N, dev)), 1, P(t_rand), 0,
                                       P(z), None, s), "stratified")
    L.check(lib.nerf_ray_features_train(P(tr.packed), P(dn), B, None, 0, P(feat), P(encd), s), "features")

    mode = os.environ.get("MODE", "plain")
    z2 = (z + 0.37).contiguous()
    rgb2, sigma2 = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
    side = torch.cuda.Stream(dev)
    ga = torch.randn(8192, 8192, device=dev)

    def fwd(fill=float("nan")):
        if mode == "scribble":
            L.check(lib.nerf_mlp_forward(P(tr.packed), P(o), P(dn), P(z2), B, N, P(feat), P(rgb2), P(sigma2), None, 0,
                                         s), "render forward")
        elif mode == "side":
            with torch.cuda.stream(side):
                torch.mm(ga, ga)
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
        save = torch.full((L.tile_rows(M), L.SAVE_ROW), fill, device=dev)
        masks = torch.full((M, L.MASK_ROW), -1 if fill != fill else int(fill), dtype=torch.int32, device=dev)
        L.check(lib.nerf_mlp_forward_train(P(tr.packed), P(o), P(dn), P(z), B, N, P(feat), P(encd), P(rgb), P(sigma),
                                           P(save), P(masks), s), "mlp_forward_train")
        torch.cuda.synchronize()
        return rgb.cpu(), sigma.cpu(), L.untile(save.cpu(), M), masks.cpu()

    ref = fwd()
    # cells the forward leaves unwritten: a second forward into buffers filled with 0 instead of NaN / -1
    zero = fwd(0.0)
    unw = torch.isnan(ref[2]) & (zero[2] == 0)
    cols = unw.any(0).nonzero().flatten().numpy()
    print(f"save cells left unwritten: {int(unw.sum())} in {len(cols)} columns; columns by segment:")
    for name, lo, hi in SEGS + [("pad", 1087, 1088)]:
        sel = cols[(cols >= lo) & (cols < hi)]
        if len(sel):
            rows = unw[:, sel].any(1).nonzero().flatten().numpy()
            print(f"  {name}: columns {sel.tolist()[:12]}{'...' if len(sel) > 12 else ''}; {len(rows)} samples, "
                  f"lane histogram {np.bincount(rows % 32, minlength=32).tolist()}")
    mw = (ref[3] == -1) & (zero[3] == 0)
    print(f"mask words left unwritten: {int(mw.sum())}; words {mw.any(0).nonzero().flatten().numpy().tolist()[:20]}")
    bad = 0
    for rep in range(1, REPS + 1):
        cur = fwd()
        diffs = []
        for name, a, b in (("rgb", ref[0], cur[0]), ("sigma", ref[1], cur[1]), ("masks", ref[3], cur[3])):
            ne = (a != b).reshape(M, -1).any(1) if name != "masks" else (a != b).any(1)
            if ne.any():
                diffs.append((name, ne))
        for name, lo, hi in SEGS:
            a, b = ref[2][:, lo:hi], cur[2][:, lo:hi]
            ne = ~((a == b) | (torch.isnan(a) & torch.isnan(b)))
            if ne.any():
                diffs.append((name, ne.any(1), ne.any(0)))
        if diffs:
            bad += 1
            print(f"rep {rep}: differs")
            for item in diffs:
                rows = item[1].nonzero().flatten().numpy()
                lanes = np.bincount(rows % 32, minlength=32)
                blocks = np.unique(rows // 32)
                msg = f"  {item[0]}: {len(rows)} samples in {len(blocks)} blocks; first blocks {blocks[:6].tolist()}; " \
                      f"lane histogram {lanes.tolist()}"
                if len(item) > 2:
                    msg += f"; features {item[2].nonzero().flatten().numpy()[:16].tolist()}"
                print(msg)
            if rep >= 1 and bad >= 3:
                break
    print(f"{bad} of {REPS} repetitions differ from the first ({os.environ.get('NERFMI_LIB') or 'in-tree'}, "
          f"mode {mode})")


if __name__ == "__main__":
    main()
