"""BASELINE config 4 on one GPU: the hotdog 800x800 frame, 64 coarse + 128 fine (H1), perturbed with
the in-kernel RNG, rendered as the G = 8 ray shards an 8-GPU node renders (frames.py, "G virtual
shards") and reassembled in ray order as the RCCL all-gather does.

* The sharded frame is bit-identical to the same frame rendered by one nerf_render_rays call: the
  in-kernel draws are keyed by the global ray index (include/nerfmi.h nerf_rng_uniforms, ray0), so
  the result does not depend on how the rays are cut (reference: the chunk loop of run.py:212-231,
  whose chunks are independent; hotdog look-at centre run.py:107).
* 4,096 rays of the frame against the oracle run on the same uniforms (regenerated with
  nerf_rng_uniforms), measured against a float64 render: the GPU's error is no worse than the fp32
  CPU oracle's own (conftest.check_no_worse_than_cpu).
Both MLP arithmetics.
"""
import pytest
import torch

from conftest import check_no_worse_than_cpu, render_h1_f64
from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu

H = W = 800
N, NF = 64, 128
SEED = 20260


@pytest.fixture(scope="module", autouse=True, params=["f16x3", "f32"])
def arith(request):
    from nerfmi import _lib as L
    prev = L.set_mlp_arith(request.param)
    yield request.param
    L.set_mlp_arith(prev)


def _uniforms(seed, first, n):
    from nerfmi import _lib as L
    out = torch.empty(n, device="cuda")
    L.check(L.load().nerf_rng_uniforms(seed, first, n, L.ptr(out), L.stream()), "nerf_rng_uniforms")
    return out


def test_hotdog_frame_as_8_virtual_shards(ref_state, app_vec, arith):
    import nerfmi
    from nerfmi import cameras, frames
    model = nerfmi.NeRF(nerfmi.Config())
    model.load_state_dict(ref_state)
    model = model.cuda().eval().requires_grad_(False)
    c2w = cameras.frame_c2w("hotdog", "circle", 0, 120)
    focal = cameras.synthetic_focal(W)
    app = app_vec.cuda()
    kw = dict(appearance_embedding=app, perturb=True, hierarchical=True, seed=SEED)
    rgb8, depth8 = frames.render_path_frames(model, [c2w], H, W, focal, 2.0, 6.0, N, NF, virtual_shards=8, **kw)
    o, d = nerfmi.get_rays(H, W, focal, c2w.float().cuda())
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    rgb1, depth1, ex = nerfmi.render_rays(model, o, d, 2.0, 6.0, N, NF, **kw)
    assert torch.equal(rgb8[0].reshape(-1, 3), rgb1), "8-shard frame differs from the one-call frame"
    assert torch.equal(depth8[0].reshape(-1), depth1[:, 0])
    # uneven shards (3 and 7 ranks: 213,334 / 91,429 rays, ragged rows) reassemble to the same bits
    for G in (3, 7):
        rgbg, depthg = frames.render_path_frames(model, [c2w], H, W, focal, 2.0, 6.0, N, NF, virtual_shards=G, **kw)
        assert torch.equal(rgbg, rgb8) and torch.equal(depthg, depth8), G
    # every ray against the frame's own size-independent properties
    assert torch.isfinite(rgb1).all() and float(rgb1.min()) >= 0 and float(rgb1.max()) <= 1
    z = ex["z_vals"]
    assert bool((z[:, 1:] >= z[:, :-1]).all())
    assert float(depth1.min()) >= 2.0 - 1e-4 and float(depth1.max()) <= 6.0 + 1e-4
    # 4096 rays against the oracle on the kernel's own uniforms (ray r: t = u(S, 64 r + s), u_f =
    # u(S ^ 0x5DEECE66D, 128 r + j)), referenced to float64
    g = torch.Generator().manual_seed(77)
    idx = torch.randperm(H * W, generator=g)[:4096]
    t_all = _uniforms(SEED, 0, H * W * N).reshape(H * W, N)
    u_all = _uniforms(SEED ^ 0x5DEECE66D, 0, H * W * NF).reshape(H * W, NF)
    t, u = t_all[idx.cuda()].cpu(), u_all[idx.cuda()].cpu()
    del t_all, u_all
    oc, dc = o[idx.cuda()].cpu(), d[idx.cuda()].cpu()
    r_ref, d_ref, ex_ref = O.render_rays_h1(ref_state, oc, dc, 2.0, 6.0, N, NF, app_vec, t, u)
    # the coarse samples are bit-exact (same uniforms, same roundings): each coarse z is in the merged row
    zg = z[idx.cuda()].cpu()
    zc = ex_ref["z_vals_coarse"]
    assert bool((zc[:, :, None] == zg[:, None, :]).any(-1).all())
    cr = ex["rgb_map_coarse"][idx.cuda()].cpu()
    err = (cr - ex_ref["rgb_map_coarse"]).abs()
    assert bool((err <= 1e-6 + 1e-4 * ex_ref["rgb_map_coarse"].abs()).all()), float(err.max())
    r64, d64 = render_h1_f64(ref_state, oc, dc, app_vec, u, t=t)
    check_no_worse_than_cpu(rgb1[idx.cuda()].cpu(), r_ref, r64, f"hotdog 8-shard {arith} rgb")
    check_no_worse_than_cpu(depth1[idx.cuda()].cpu(), d_ref, d64, f"hotdog 8-shard {arith} depth")
    psnr = -10 * torch.log10(((rgb1[idx.cuda()].cpu() - r_ref) ** 2).mean())
    assert float(psnr) > 80, float(psnr)
