"""Render-MLP time per sample against launch size: nerf_mlp_forward (the render kernel of the loaded
library) on R rays x 64 samples for R from 1K to 1M, each size launched back to back for >= 1 s
(after a 1 s warm-up at that size), timed by HIP events around the timed launches.  Prints one JSON
line per size.  NERFMI_LIB selects the library (A/B of the 16x16x32 kernel against round 5's 32x32).
Diagnostic, not a test."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import nerfmi  # noqa: E402
from nerfmi import _lib as L  # noqa: E402
from nerfmi.ray_utils import linspace_table  # noqa: E402
from nerfmi.train import Trainer  # noqa: E402


def main():
    lib, P, s = L.load(), L.ptr, L.stream()
    dev = L.device()
    torch.manual_seed(0)
    tr = Trainer(nerfmi.Config())
    L.check(lib.nerf_pack_weights(tr.param_ptrs, P(tr.packed), s), "pack")   # (a Trainer packs in its step)
    N = 64
    for R in (1024, 4096, 16384, 65536, 262144, 1048576):
        M = R * N
        g = torch.Generator().manual_seed(R)
        o = (torch.randn(R, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
        d = torch.randn(R, 3, generator=g).to(dev)
        d[:, 2] = -d[:, 2].abs() - 1.0
        t_rand = torch.rand(R, N, generator=g).to(dev)
        dn, z = torch.empty(R, 3, device=dev), torch.empty(R, N, device=dev)
        feat, encd = torch.empty(R, 256, device=dev), torch.empty(R, 32, device=dev)
        L.check(lib.nerf_normalize_dirs(P(d), R, P(dn), s), "normalize")
        L.check(lib.nerf_sample_stratified(P(o), P(dn), R, tr.near, tr.far, N, P(linspace_table(N, dev)), 1,
                                           P(t_rand), 0, P(z), None, s), "stratified")
        L.check(lib.nerf_ray_features_train(P(tr.packed), P(dn), R, None, 0, P(feat), P(encd), s), "features")
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)

        def launch():
            L.check(lib.nerf_mlp_forward(P(tr.packed), P(o), P(dn), P(z), R, N, P(feat), P(rgb), P(sigma), None, 0, s),
                    "render forward")
        t0 = time.time()
        while time.time() - t0 < 1.0:
            launch()
            torch.cuda.synchronize()
        n = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.time()
        e0.record()
        while time.time() - t0 < 1.0 or n < 5:
            for _ in range(5):
                launch()
            n += 5
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(json.dumps({"lib": os.path.basename(os.environ.get("NERFMI_LIB") or "in-tree"), "rays": R,
                          "samples": M, "ms_per_launch": round(ms, 4), "ns_per_sample": round(ms * 1e6 / M, 4),
                          "tflops": round(M * 1048832 / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
