"""The in-kernel RNG (csrc/common.h hash_uniform) that draws the stratified jitter and the
inverse-CDF uniforms when no explicit uniforms are passed: the path bench.py and run.py use.

1. The generator nerf_rng_uniforms exposes is the one the render path uses: a render keyed by
   `seed` equals, bit for bit, the same render with t_rand = u(seed, r*N+s) and
   u_rand = u(seed ^ 0x5DEECE66D, r*Nf+j) passed explicitly (render.py's draw order).
2. Its distribution, on 2^24 draws per stream: Kolmogorov-Smirnov against U(0,1) at the 1%
   level, lag-1 correlation along a ray's samples and across neighbouring rays below 1e-3
   (4 sigma at this n), the two streams of one seed and the streams of adjacent seeds (frames,
   shards) uncorrelated below 1e-3, and pairs (u_i, u_i+1) uniform on a 64x64 grid (chi-square
   within 5 sigma of its 4095 degrees of freedom)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEY = 0x5DEECE66D
N_DRAWS = 1 << 24


def uniforms(seed, n, first=0):
    from nerfmi import _lib as L
    out = torch.empty(n, device="cuda")
    L.check(L.load().nerf_rng_uniforms(seed & (2 ** 64 - 1), first, n, L.ptr(out), L.stream()), "rng")
    return out


def corr(a, b):
    a = a.double().flatten() - a.double().mean()
    b = b.double().flatten() - b.double().mean()
    return float((a * b).sum() / torch.sqrt((a * a).sum() * (b * b).sum()))


def test_render_path_draws_are_the_exposed_generator(ref_state, app_vec):
    import nerfmi
    from nerfmi import cameras
    m = nerfmi.NeRF(nerfmi.Config())
    m.load_state_dict(ref_state)
    m = m.cuda().eval().requires_grad_(False)
    c2w = cameras.frame_c2w("chair").cuda()
    o, d = nerfmi.get_rays(800, 800, cameras.synthetic_focal(800), c2w)
    o, d = o[380:412, 300:500].reshape(-1, 3), d[380:412, 300:500].reshape(-1, 3)
    B, seed = o.shape[0], 123456789
    a = nerfmi.render_rays(m, o, d, 2.0, 6.0, 64, 128, appearance_embedding=app_vec.cuda(), perturb=True,
                           hierarchical=True, seed=seed)
    t = uniforms(seed, B * 64).reshape(B, 64)
    u = uniforms(seed ^ KEY, B * 128).reshape(B, 128)
    b = nerfmi.render_rays(m, o, d, 2.0, 6.0, 64, 128, appearance_embedding=app_vec.cuda(), perturb=True,
                           hierarchical=True, t_rand=t, u_rand=u)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2]["z_vals"], b[2]["z_vals"])
    # the stratified entry point alone
    dn = torch.nn.functional.normalize(d, dim=-1)
    z1, _ = nerfmi.sample_stratified(o, dn, 2.0, 6.0, 64, seed=seed)
    z2, _ = nerfmi.sample_stratified(o, dn, 2.0, 6.0, 64, perturb=True, t_rand=t)
    assert torch.equal(z1, z2)
    # first/offset addressing
    assert torch.equal(uniforms(seed, 1000, first=5000), uniforms(seed, 6000)[5000:])


@pytest.mark.parametrize("seed", [0, 1, 123456789, 2 ** 63 + 17])
def test_uniform_ks_and_range(seed):
    for key in (seed, seed ^ KEY):
        x = uniforms(key, N_DRAWS)
        assert float(x.min()) >= 0.0 and float(x.max()) < 1.0
        xs = torch.sort(x).values.double()
        n = xs.numel()
        i = torch.arange(1, n + 1, device=xs.device, dtype=torch.float64)
        D = max(float((i / n - xs).max()), float((xs - (i - 1) / n).max()))
        assert D < 1.63 / math.sqrt(n), (key, D)            # KS at alpha = 0.01
        assert abs(float(x.double().mean()) - 0.5) < 5 * math.sqrt(1 / 12 / n)


@pytest.mark.parametrize("N", [64, 128])
def test_no_correlation_along_or_across_rays(N):
    x = uniforms(777, N_DRAWS).reshape(-1, N)                 # ray-major, as r*N + s
    assert abs(corr(x[:, :-1], x[:, 1:])) < 1e-3              # lag 1 along a ray's samples
    assert abs(corr(x[:-1], x[1:])) < 1e-3                    # same sample, neighbouring rays
    assert abs(corr(x[:, :-2], x[:, 2:])) < 1e-3              # lag 2


def test_streams_are_separate():
    s = 987654321
    a = uniforms(s, N_DRAWS)
    assert abs(corr(a, uniforms(s ^ KEY, N_DRAWS))) < 1e-3    # stratified vs inverse-CDF key
    assert abs(corr(a, uniforms(s + 1, N_DRAWS))) < 1e-3      # adjacent seeds (frames, shards)
    assert abs(corr(a[1:], uniforms(s + 1, N_DRAWS)[:-1])) < 1e-3
    assert not torch.equal(a[:1000], uniforms(s + 1, 1000))


def test_pairs_fill_the_unit_square():
    x = uniforms(31337, N_DRAWS)
    bins = 64
    cell = (torch.clamp((x[:-1] * bins).long(), max=bins - 1) * bins
            + torch.clamp((x[1:] * bins).long(), max=bins - 1))
    counts = torch.bincount(cell, minlength=bins * bins).double()
    exp = (x.numel() - 1) / (bins * bins)
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    dof = bins * bins - 1
    assert abs(chi2 - dof) < 5 * math.sqrt(2 * dof), chi2
