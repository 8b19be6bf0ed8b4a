"""A/B timing of MLP kernel builds (make -C <pkg> variants) in ONE process, interleaved rounds.

Each variant library is loaded with ctypes (RTLD_LOCAL) and runs nerf_mlp_forward on the same
inputs (the coarse pass of an 800x800 frame: 640,000 rays x 64 samples); the kernel is timed
with events on the launch stream.  Also checks every variant's output against the in-tree
library's (max relative difference)."""
import ctypes, glob, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import nerfmi
from nerfmi import _lib, cameras

PKG = os.path.dirname(_lib.LIB_PATH)
libs = {"tree": _lib.load()}
for p in sorted(glob.glob(os.path.join(PKG, "build", "variants", "libnerfmi_*.so"))):
    L = ctypes.CDLL(p)
    for name, (res, args) in _lib._SIGNATURES.items():
        if not hasattr(L, name):
            continue
        f = getattr(L, name); f.restype = res; f.argtypes = args
    libs[os.path.basename(p)[10:-3]] = L
torch.manual_seed(0)
model = nerfmi.NeRF(nerfmi.Config()).cuda().eval()
packed = model.packed_weights()
torch.manual_seed(1)
app = torch.randn(1, 32).cuda()
o, d = nerfmi.get_rays(800, 800, cameras.synthetic_focal(800), cameras.frame_c2w("chair").cuda())
o = o.reshape(-1, 3).contiguous(); d = torch.nn.functional.normalize(d.reshape(-1, 3), dim=-1).contiguous()
B, N = o.shape[0], int(os.environ.get("NSAMP", "64"))
z, _ = nerfmi.sample_stratified(o, d, 2.0, 6.0, N, perturb=True, seed=3)
z = z.contiguous()
P = _lib.ptr
feat = torch.empty(B, 256, device="cuda")
s = _lib.stream()
_lib.check(libs["tree"].nerf_ray_features(P(packed), P(d), B, P(app), 1, P(feat), s), "feat")
outs = {k: (torch.empty(B * N, 3, device="cuda"), torch.empty(B * N, device="cuda")) for k in libs}
times = {k: [] for k in libs}
rounds = int(os.environ.get("ROUNDS", "4"))
for r in range(rounds + 1):
    for k, L in libs.items():
        rgb, sig = outs[k]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(L.nerf_mlp_forward(P(packed), P(o), P(d), P(z), B, N, P(feat), P(rgb), P(sig), None, 0, s), k)
        e1.record()
        torch.cuda.synchronize()
        if r > 0:
            times[k].append(e0.elapsed_time(e1))
ref_rgb, ref_sig = outs["tree"]
res = {}
for k in libs:
    t = sorted(times[k])
    tf = B * N * 1_048_832 / (t[len(t) // 2] * 1e-3) / 1e12
    rgb, sig = outs[k]
    dr = float(((rgb - ref_rgb).abs() / ref_rgb.abs().clamp_min(1e-6)).max())
    res[k] = {"median_ms": t[len(t) // 2], "min_ms": t[0], "tflops": tf, "frac_f32_peak": tf / 157.3, "max_rel_vs_tree_rgb": dr}
    print(k, json.dumps(res[k]), flush=True)
