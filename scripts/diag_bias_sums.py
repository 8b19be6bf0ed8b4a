"""Diagnostic (GPU): where the f16x3 training path's bias-gradient error comes from.

On 8,192 samples (seed-0 weights, random rays and upstream gradients), per layer l: the bias gradient
sum_m d pre_l[m] (a) from the data-gradient rows nerf_mlp_backward wrote, summed in float64 on the
host, and (b) from nerf_param_grads (the weight-gradient kernels' bias column + chunk reduction),
each as rel error against float64 autograd; and the rows' own rel-L2 plus their mean signed relative
error sign(x) (gpu - x) / |x| (a systematic shrink or growth of the rows shows up there)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from nerfmi import _lib as L
    from oracle import nerf_oracle as O
    from test_gpu_train import _draw, _mlp_forward_backward, packed_of, rel_l2
    ref = O.random_state(0)
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0]
    lib, dev = L.load(), L.device()
    for arith in ("f16x3", "f32"):
        L.set_mlp_arith(arith)
        R, N = 512, 16
        draw = _draw(R, N, 5)
        r = _mlp_forward_backward(ref, app, R, N, draw=draw)
        M = R * N
        save, grad = r["save_tiled"].to(dev), r["grad_tiled"].to(dev)
        packed, _, ts = packed_of(ref, dev)
        grads = [torch.zeros_like(t) for t in ts]
        arr = (ctypes.c_void_p * 24)(*[t.data_ptr() for t in grads])
        a = app.reshape(1, 32).to(dev).contiguous()
        dapp = torch.empty(1, 32, device=dev)
        ws = torch.empty(lib.nerf_param_grads_workspace_bytes(M), dtype=torch.uint8, device=dev)
        L.check(lib.nerf_param_grads(L.ptr(save), L.ptr(grad), M, N, L.ptr(a), 1, L.ptr(packed), arr, L.ptr(dapp),
                                     L.ptr(ws), ws.numel(), L.stream()), "param_grads")
        torch.cuda.synchronize()
        rows = np.asarray(r["grad"], np.float64)
        print(f"== {arith}")
        for l in range(7, -1, -1):
            exp = r["pres"][l].grad.numpy()
            got = rows[:, 256 * l:256 * (l + 1)]
            b64 = exp.sum(0)
            sym = np.sign(exp) * (got - exp) / np.maximum(np.abs(exp), 1e-30)
            keep = np.abs(exp) > 1e-3 * np.abs(exp).max()
            bias_k = grads[2 * l + 1].cpu().double().numpy()
            err = got - exp
            mean_err = err.mean(0) / (np.sqrt((exp ** 2).mean(0)) + 1e-30)       # per column, in row-rms units
            print(f"  l={l}: rows rel-L2 {rel_l2(got, exp):.3g}  mean signed rel {sym[keep].mean():+.3g}  "
                  f"mean err/rms per column: median {np.median(mean_err):+.3g} max|.| {np.abs(mean_err).max():.3g} "
                  f"(random would be ~{rel_l2(got, exp) / np.sqrt(len(exp)):.2g}) "
                  f"| bias from rows (f64 sum) {rel_l2(got.sum(0), b64):.3g}  bias from param_grads "
                  f"{rel_l2(bias_k, b64):.3g}  weight {rel_l2(grads[2 * l].cpu().numpy(), r['st64'][f'pts_linears.{l}.weight'].grad.numpy()):.3g}")


if __name__ == "__main__":
    main()
