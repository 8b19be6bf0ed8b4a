"""Where two identically seeded trainers (tests/test_gpu_train.py::test_training_is_deterministic's
setup) first diverge: per step, per-column bit checksums of the training workspace's save rows, mask
rows and gradient rows (nerf_train_forward / nerf_train_backward's carve, csrc/train.hip train_carve),
the parameter gradients and the parameters.  NERFMI_LIB selects the library.  Diagnostic, not a test."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import nerfmi  # noqa: E402
from nerfmi import _lib as L  # noqa: E402
from nerfmi.dataset import SyntheticNeRFDataset  # noqa: E402
from nerfmi.train import Trainer  # noqa: E402

STEPS = int(os.environ.get("STEPS", "6"))
SEGS = [("h%d" % j, o, o + 256) for j, o in enumerate([0, 256, 512, 768, 1088, 1344, 1600, 1856])] + \
       [("enc_x", 1024, 1088), ("enc_d", 2112, 2144), ("r_dir", 2144, 2272), ("hd", 2272, 2400)]


def carve(B, N):
    """Byte offsets of train_carve's regions: dirs z feat encd rgb sigma maps dsigma drgb sq_err save masks grad."""
    M, MT = B * N, L.tile_rows(B * N)
    sizes = [B * 3, B * N, B * 256, B * 32, M * 3, M, B * 4, M, M * 3, B, MT * L.SAVE_ROW, M * L.MASK_ROW,
             MT * L.GRAD_ROW]
    off, at = [], 0
    for sz in sizes:
        off.append(at)
        at += (sz * 4 + 255) & ~255
    return dict(zip(["dirs", "z", "feat", "encd", "rgb", "sigma", "maps", "dsig", "drgb", "sqe", "save", "masks",
                     "grad"], off)), M, MT


def colsum(t, ncol):
    """Per-column sum of the int32 bit patterns (int64)."""
    return t.view(torch.int32).reshape(-1, ncol).to(torch.int64).sum(0).cpu().numpy()


def run():
    cfg = nerfmi.Config()
    np.random.seed(0)
    torch.manual_seed(0)
    ds = SyntheticNeRFDataset(cfg, n_images=3, H=96, W=96)
    torch.manual_seed(0)
    tr = Trainer(cfg, appearance_embeddings=ds.appearance_embeddings)
    recs = []
    for i in range(STEPS):
        b = ds.get_rays(batch_size=4096)
        loss, _ = tr.forward_backward(b["rays_o"], b["rays_d"], b["rgb"], b["appearance_idx"], seed=i + 1)
        torch.cuda.synchronize()
        ws = tr._ws
        off, M, MT = carve(4096, cfg.num_samples)
        f32 = lambda name, n: ws[off[name]: off[name] + n * 4].view(torch.float32)  # noqa: E731
        rec = {"loss": float(loss),
               "rgb": colsum(f32("rgb", M * 3), 3), "sigma": colsum(f32("sigma", M), 1),
               "dsig": colsum(f32("dsig", M), 1), "drgb": colsum(f32("drgb", M * 3), 3),
               "save": colsum(f32("save", MT * L.SAVE_ROW).reshape(MT // 32, L.SAVE_ROW // 8, 32, 8)
                              .permute(0, 2, 1, 3).reshape(MT, L.SAVE_ROW), L.SAVE_ROW),
               "masks": colsum(f32("masks", M * L.MASK_ROW), L.MASK_ROW),
               "grad_rows": colsum(f32("grad", MT * L.GRAD_ROW).reshape(MT // 32, L.GRAD_ROW // 8, 32, 8)
                                   .permute(0, 2, 1, 3).reshape(MT, L.GRAD_ROW), L.GRAD_ROW),
               "param_grad": [colsum(tr.view(tr.grad, k).reshape(-1), 1)[0] for k in range(25 if tr.n_images else 24)],
               "packed": colsum(tr.packed, 1), "packedT": colsum(tr.packedT, 1)}
        tr.all_reduce()
        tr.optimizer_step()
        torch.cuda.synchronize()
        rec["flat"] = colsum(tr.flat, 1)
        recs.append(rec)
    return recs


def main():
    a, b = run(), run()
    for i, (ra, rb) in enumerate(zip(a, b)):
        diffs = []
        for k in ra:
            va, vb = np.asarray(ra[k]), np.asarray(rb[k])
            if not np.array_equal(va, vb):
                cols = np.nonzero(va != vb)[0] if va.ndim else []
                extra = ""
                if k == "save":
                    extra = " segments " + ",".join(sorted({n for n, lo, hi in SEGS for c in cols if lo <= c < hi}))
                diffs.append(f"{k} ({len(cols)} columns: {list(cols[:10])}{extra})")
        print(f"step {i}: " + ("identical" if not diffs else "; ".join(diffs)))
        if diffs and i >= 1 and all("identical" not in d for d in diffs) and len(diffs) > 8:
            break
    print(f"library: {os.environ.get('NERFMI_LIB') or 'in-tree'}")


if __name__ == "__main__":
    main()
