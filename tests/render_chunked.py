"""Child of tests/test_gpu_parity.py::test_render_chunked_matches_one_launch: renders the test's
batch in this process, whose NERFMI_MAX_LAUNCH_SAMPLES (set by the parent) makes nerf_render_rays
and nerf_mlp_forward split the call into ray chunks, and saves the outputs for the parent."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def render(out_path=None, arith=None):
    import nerfmi
    if arith:
        nerfmi.set_mlp_arith(arith)
    torch.manual_seed(0)
    model = nerfmi.NeRF(nerfmi.Config()).cuda().eval()
    g = torch.Generator().manual_seed(7)
    B = 3000
    o = torch.randn(B, 3, generator=g) * 0.2
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1)
    app = torch.randn(B, 32, generator=g)                  # one appearance row per ray
    outs = {}
    with torch.no_grad():
        for staged in (False, True):
            rgb, depth, ex = nerfmi.render_rays(model, o.cuda(), d.cuda(), 2.0, 6.0, 64, 128, appearance_embedding=app.cuda(),
                                                perturb=True, hierarchical=True, seed=1234, ray_offset=5, staged=staged)
            for k, v in (("rgb", rgb), ("depth", depth), ("weights", ex["weights"]), ("z", ex["z_vals"]),
                         ("rgb_c", ex["rgb_map_coarse"])):
                outs[f"{k}_{int(staged)}"] = v.cpu()
    if out_path:
        torch.save(outs, out_path)
    return outs


if __name__ == "__main__":
    render(sys.argv[1], sys.argv[2])
