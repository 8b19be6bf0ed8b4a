"""Error of the GPU MLP and of the CPU reference arithmetic, each against an fp64 evaluation."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import nerfmi
from oracle import nerf_oracle as O

st = O.random_state(0)
st64 = {k: v.double() for k, v in st.items()}
m = nerfmi.NeRF(nerfmi.Config()); m.load_state_dict(st); m = m.cuda().eval()
torch.manual_seed(1); app = torch.randn(100, 32)[0]
torch.manual_seed(5)
x = torch.randn(65536, 3) * 1.5
d = torch.nn.functional.normalize(torch.randn(65536, 3), dim=-1)
with torch.no_grad():
    rg, sg = m(x.cuda(), d.cuda(), app.cuda())
rc, sc = O.nerf_forward(st, x, d, app)
r64, s64 = O.nerf_forward(st64, x.double(), d.double(), app.double())
for name, a, b, ref in (("rgb", rg.cpu().double(), rc.double(), r64), ("sigma", sg.cpu().double(), sc.double(), s64)):
    den = ref.abs().clamp_min(1e-6)
    print(f"{name}: gpu vs fp64 max rel {float(((a-ref).abs()/den).max()):.3e} rms rel {float(((a-ref)/den).pow(2).mean().sqrt()):.3e} | "
          f"cpu vs fp64 max rel {float(((b-ref).abs()/den).max()):.3e} rms rel {float(((b-ref)/den).pow(2).mean().sqrt()):.3e} | "
          f"gpu vs cpu max rel {float(((a-b).abs()/den).max()):.3e}")
