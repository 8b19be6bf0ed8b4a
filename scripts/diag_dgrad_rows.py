"""Diagnostic (GPU): per-layer error of the data-gradient rows d pre_l (nerf_mlp_backward) against float64.

Seed-0 and adversarial weights (tests/test_gpu_accuracy.py), 8,192 samples on random rays: rel-L2 of
the GPU's rows, of the f16x3 emulation's (f16x3_gradient_emulation below: the
kernel's splits, exact products) and of the fp32 CPU autograd's, each against float64 autograd, per
layer (the sample masks of the GPU forward; rays with a float64 pre-activation at a kink dropped)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle import nerf_oracle as O  # noqa: E402


def _split16(x, s):
    """The kernels' split of x (fp32) at the power-of-two scale s (stream16.h split_into): x s = hi +
    lo, both f16; returned as float64 for exact products."""
    xs = x.float() * s.float()
    hi = xs.half()
    lo = (xs - hi.float()).half()
    return hi.double(), lo.double()


def _pow2_scale(m):
    """stream16.h pow2_scale: 2^(14 - e) for m < 2^e (frexp)."""
    _, e = torch.frexp(m.float())
    return torch.ldexp(torch.ones_like(m, dtype=torch.float32), (14 - e.clamp(-100, 100)).to(torch.int32))


def _f16x3_rows_times(g, w):
    """d_in = g @ w (g: M x N gradient rows, w: N x K weight) in the data-gradient kernels' split-f16
    arithmetic: w split at its matrix scale (2^(14-e), e from max|w|), each row of g at its own scale,
    hi(w)hi(g) + hi(w)lo(g) + lo(w)hi(g) (lo lo dropped), exact products, one rounding to fp32."""
    sw = _pow2_scale(w.abs().max())
    sg = _pow2_scale(g.abs().amax(dim=1, keepdim=True))
    wh, wl = _split16(w, sw)
    gh, gl = _split16(g, sg)
    return ((gh @ wh + gl @ wh + gh @ wl) / (sw.double() * sg.double())).float()


def f16x3_gradient_emulation(st, x, d, app, masks, g_rgb, g_sig, rows=False):
    """Every parameter gradient with the data-gradient chain in the f16x3 arithmetic of
    mlp_backward16_bound_kernel (_f16x3_rows_times per layer: d h_{l-1} = d pre_l W_l), everything else
    in float64 on the given ReLU branches: the error this arithmetic carries by itself, against which
    the GPU's f16x3 gradients are held (test_gradients_vs_float64)."""
    sd = {k: v.double() for k, v in st.items()}
    ins = []
    with torch.no_grad():
        class Rec:
            def __getattr__(self, k):
                return getattr(torch.nn.functional, k)

            def linear(self, a, w, b=None):
                ins.append(a)
                return torch.nn.functional.linear(a, w, b)
        saved, O.F = O.F, Rec()
        try:
            rgb, sigma = O.nerf_forward(sd, x.double(), d.double(), app.double(),
                                        relu=lambda pre, i: pre * masks[i].double())
        finally:
            O.F = saved
    # ins: pts_linears 0..7, density_head, dir_linear, appearance_projection, rgb_linear
    h_in, hd_in, dir_in, app_in = ins[:8], ins[11], ins[9], ins[10]
    f32 = {k: v.float() for k, v in st.items()}
    dv = g_rgb.float() * (rgb.float() * (1.0 - rgb.float()))                     # sigmoid'
    dsp = g_sig.float() * masks[8].float()                                       # ReLU(density)'
    dhd = dv @ f32["rgb_linear.weight"]                                          # M x 128, fp32 VALU
    dpre = {"dir": dhd * masks[9].float()}
    dh = _f16x3_rows_times(dpre["dir"], f32["dir_linear.weight"][:, :256]) + dsp * f32["density_head.weight"]
    for l in range(7, -1, -1):
        dpre[l] = dh * masks[l].float()
        if l:
            dh = _f16x3_rows_times(dpre[l], f32[f"pts_linears.{l}.weight"][:, :256])
    out = {}
    for l in range(8):
        out[f"pts_linears.{l}.weight"] = dpre[l].double().T @ h_in[l]
        out[f"pts_linears.{l}.bias"] = dpre[l].double().sum(0)
    out["density_head.weight"] = dsp.double().T @ ins[8]
    out["density_head.bias"] = dsp.double().sum(0)
    out["dir_linear.weight"] = dpre["dir"].double().T @ dir_in
    out["dir_linear.bias"] = dpre["dir"].double().sum(0)
    out["appearance_projection.weight"] = dhd.double().T @ app_in
    out["appearance_projection.bias"] = dhd.double().sum(0)
    out["rgb_linear.weight"] = dv.double().T @ hd_in
    out["rgb_linear.bias"] = dv.double().sum(0)
    return (out, dpre) if rows else out




def main():
    from nerfmi import _lib
    from test_gpu_accuracy import adversarial_state
    from test_gpu_train import _draw, _mlp_forward_backward, rel_l2
    ref = O.random_state(0)
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0]
    _lib.set_mlp_arith(os.environ.get("DIAG_ARITH", "f16x3"))
    for which, st in (("seed0", ref), ("adversarial", adversarial_state(ref))):
        R, N = 512, 16
        draw = _draw(R, N, 5)
        r = _mlp_forward_backward(st, app, R, N, draw=draw)
        o, d, z, g_rgb, g_sig = draw
        pts, dexp = r["pts"], r["dexp"]
        save = r["save"]
        h_at = [l * 256 if l < 4 else 1088 + (l - 4) * 256 for l in range(8)]
        masks = [torch.from_numpy(save[:, a:a + 256].numpy() > 0) if hasattr(save, "numpy") else save[:, a:a + 256] > 0
                 for a in h_at]
        masks.append((r["sigma"] > 0).reshape(-1, 1))
        masks.append(torch.as_tensor(np.asarray(save[:, 2144:2272]) > 0))
        _, emul = f16x3_gradient_emulation(st, pts.float(), dexp.float(), app, masks, g_rgb, g_sig.reshape(-1, 1),
                                           rows=True)
        st32 = {k: v.float().clone().requires_grad_(True) for k, v in st.items()}
        pres32 = []
        rgb32, sig32 = O.nerf_forward(st32, pts.float(), dexp.float(), app.float(), keep=pres32)
        for t in pres32:
            t.retain_grad()
        ((rgb32 * g_rgb).sum() + (sig32[:, 0] * g_sig).sum()).backward()
        grad = np.asarray(r["grad"])
        print(f"== {which}")
        for l in range(7, -1, -1):
            exp = r["pres"][l].grad.numpy()
            print(f"  d pre_{l}: gpu {rel_l2(grad[:, 256 * l:256 * (l + 1)], exp):.3g}  emul "
                  f"{rel_l2(emul[l].double().numpy(), exp):.3g}  cpu32 {rel_l2(pres32[l].grad.double().numpy(), exp):.3g}")


if __name__ == "__main__":
    main()
