"""Diagnostic (host): the composite forward on inputs saved by DIAG_SAVE=<dir> python scripts/diag_dir_grads.py
(the GPU's own rgb / sigma / z of one training batch): the GPU kernel's rgb_map, torch's fp32 composite and
an emulation of the kernel (correctly rounded exp, double transmittance products) or with torch's exp, each
against float64 on the same inputs.  torch's CPU float exp is host-dependent."""
import sys, numpy as np, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import nerf_oracle as O
d = np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/r05/diag/composite_inputs_f16x3.npz')
B, N = 512, 64
rgb = torch.from_numpy(d['rgb']).reshape(B, N, 3); sigma = torch.from_numpy(d['sigma']).reshape(B, N, 1); z = torch.from_numpy(d['z'])
def bias(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64); return (a - b).mean() / np.sqrt((b ** 2).mean())
def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64); return np.linalg.norm(a - b) / np.linalg.norm(b)
r64, _, _ = O.composite(rgb.double(), sigma.double(), z.double())
r32, _, _ = O.composite(rgb, sigma, z)
print("sigma stats: zero frac %.2f  median %.3g  max %.3g" % ((d['sigma'] == 0).mean(), np.median(d['sigma']), d['sigma'].max()))
print("torch fp32 rgb_map rel %.3g bias %+.3g" % (rel(r32, r64), bias(r32, r64)))
print("gpu kernel  rgb_map rel %.3g bias %+.3g" % (rel(d['rgb_map'], r64), bias(d['rgb_map'], r64)))
zn = d['z']; sg = d['sigma'].reshape(B, N); c = d['rgb'].reshape(B, N, 3)
dist = np.concatenate([zn[:, 1:] - zn[:, :-1], np.full((B, 1), 1e-3, np.float32)], 1).astype(np.float32)
x = (-sg * dist).astype(np.float32)
for name, e in (("expf_rn", np.exp(x.astype(np.float64)).astype(np.float32)), ("torch exp", torch.exp(torch.from_numpy(x)).numpy())):
    alpha = (np.float32(1) - e).astype(np.float32)
    f = ((np.float32(1) - alpha) + np.float32(1e-10)).astype(np.float32)
    T = np.cumprod(np.concatenate([np.ones((B, 1)), f[:, :-1].astype(np.float64)], 1), 1).astype(np.float32)
    w = (alpha * T).astype(np.float32)
    rm = ((w[..., None] * c).astype(np.float32).astype(np.float64)).sum(1).astype(np.float32)
    print("emul %-9s rgb_map rel %.3g bias %+.3g   == kernel: %.3f" % (name, rel(rm, r64), bias(rm, r64), (rm == d['rgb_map']).mean()))
