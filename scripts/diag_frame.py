"""Diagnose full-frame parity outliers: which rays, and whether they come from the fine z or the MLP."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, numpy as np
import nerfmi
from nerfmi import cameras
from oracle import nerf_oracle as O

st = O.random_state(0)
m = nerfmi.NeRF(nerfmi.Config()); m.load_state_dict(st); m = m.cuda().eval()
torch.manual_seed(1); app = torch.randn(100, 32)[0]
c2w = cameras.frame_c2w("chair").cuda()
o, d = nerfmi.get_rays(800, 800, cameras.synthetic_focal(800), c2w)
o, d = o.reshape(-1, 3), d.reshape(-1, 3)
torch.manual_seed(10)
u = torch.rand(o.shape[0], 128)
rgb, depth, ex = nerfmi.render_rays(m, o, d, 2.0, 6.0, 64, 128, appearance_embedding=app.cuda(), perturb=False,
                                    hierarchical=True, u_rand=u)
idx = torch.randperm(o.shape[0])[:4096]
r_ref, d_ref, exr = O.render_rays_h1(st, o[idx].cpu(), d[idx].cpu(), 2.0, 6.0, 64, 128, app, None, u[idx])
g = rgb[idx].cpu()
err = (g - r_ref).abs()
tol = 1e-6 + 1e-4 * r_ref.abs()
bad = (err > tol).any(-1)
print("bad rays", int(bad.sum()), "of", len(idx))
rel = (err / r_ref.abs().clamp_min(1e-12))
print("max rel err", float(rel.max()), "median rel", float(rel.median()), "max abs", float(err.max()))
print("rgb magnitude: mean", float(r_ref.mean()), "min", float(r_ref.min()))
for i in torch.nonzero(bad).flatten()[:5].tolist():
    ray = idx[i]
    zg = ex["z_vals"][ray].cpu(); zr = exr["z_vals"][i]
    print(f"ray {int(ray)}: gpu {g[i].tolist()} ref {r_ref[i].tolist()} | coarse gpu {ex['rgb_map_coarse'][ray].tolist()} ref {exr['rgb_map_coarse'][i].tolist()}")
    print("   z max rel diff", float(((zg - zr).abs() / zr).max()), "n differ", int((zg != zr).sum()))
    # fine pass through the oracle with the GPU's z_all: isolates the MLP from the resample
    zz = zg[None]
    dn = O.normalize(d[ray:ray+1].cpu())
    pts = o[ray:ray+1].cpu()[..., None, :] + dn[..., None, :] * zz[..., :, None]
    rr, dd, _ = O._pass(st, pts, dn, zz, app)
    print("   oracle MLP on gpu z:", rr[0].tolist())
# coarse-only parity over the same rays
r_c, _, _ = O.volume_render(st, o[idx].cpu(), d[idx].cpu(), 2.0, 6.0, 64, app)
gc = ex["rgb_map_coarse"][idx].cpu()
e = (gc - r_c).abs(); t = 1e-6 + 1e-4 * r_c.abs()
print("coarse bad rays", int((e > t).any(-1).sum()), "max rel", float((e / r_c.abs().clamp_min(1e-12)).max()))
