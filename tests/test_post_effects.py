"""Depth-aware post effects: nerfmi.PostProcessor's GPU kernels
(csrc/effects.hip) against oracle/post_oracle.py and, for Fog, against the reference's own outputs.

Fog is pinned by fixture F9 (tests/golden/f9_fog.npz, tests/golden/make_post_golden.py): the
reference's `_effect_fog` (src/post_processor.py:451-493, numpy only) compiled by itself from the
module's source and run on synthetic frames here, since the module as a whole imports cv2 and
tkinter, which are absent.  The oracle equals F9 bit for bit; the kernel equals it except where
the reference's `adjusted ** 3.0` (numpy's float32 SIMD pow, faithfully rounded and
host-dependent) differs from the correctly rounded cube the kernel computes, and there by at most
one count.  Toon stays unpinned against the reference: its edge steps are cv2 calls
(bilateralFilter, Sobel, dilate, cvtColor, Laplacian), restated in the oracle from OpenCV 4's
algorithms.  Tolerances: none beyond the documented cube step.  Every operation is an IEEE
float32 operation in the reference's order on both sides (-ffp-contract=off on the device; the
bilateral LUT's exp in double, then rounded), so Toon is compared bit for bit with the oracle,
and so is Fog with the oracle's cube_rn form.
"""
import os

import numpy as np
import pytest
import torch

from oracle import post_oracle as P

F9 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "f9_fog.npz")
F9_CASES = ["norm", "raw", "chan", "edges", "start0", "start35", "none"]


def f9_case(name):
    z = np.load(F9)
    depth = z[f"{name}_depth"] if f"{name}_depth" in z else None
    differs = z[f"{name}_cube_differs"] if depth is not None else None
    return z[f"{name}_img"], depth, float(z[f"{name}_start"]), z[f"{name}_out"], differs


def scene(H=96, W=120, seed=0):
    """A synthetic frame: smooth colours, a box in front of a slanted background (depth edges)."""
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([(xx / W) * 255, (yy / H) * 255, 128 + 100 * np.sin(xx / 7 + yy / 11)], -1)
    img = np.clip(img + g.normal(0, 4, img.shape), 0, 255).astype(np.uint8)
    depth = (3.0 + 0.4 * xx / W + 0.02 * np.sin(yy / 9)).astype(np.float32)
    depth[H // 4: 3 * H // 4, W // 3: 2 * W // 3] = 2.2
    return img, depth


# ------------------------------------------------------------------------------ CPU (oracle)
def test_oracle_fog_limits():
    img, depth = scene()
    out = P.fog(img, P.depth_normalize(depth), fog_start=0.1)
    near = P.depth_normalize(depth) <= 0.1 + 1e-6           # no fog factor: pure white fog
    assert np.all(out[near] == 255)
    far = P.fog(img, np.ones_like(depth), fog_start=0.1)     # factor 0.3: 0.3 img + 0.7 * 255
    exp = np.clip(img.astype(np.float32) * np.float32(0.3) + np.float32(255) * np.float32(0.7), 0, 255).astype(np.uint8)
    assert np.array_equal(far, exp)
    none = P.fog(img, None)
    assert np.array_equal(none, np.clip(img.astype(np.float32) * np.float32(0.05) + np.float32(242.25), 0,
                                        255).astype(np.uint8))


def test_oracle_bilateral_and_sobel():
    f = np.full((12, 13), 0.25, np.float32)
    assert np.array_equal(P.bilateral_32f(f), f)                       # constant image is copied
    ramp = np.tile(np.linspace(0, 1, 40, dtype=np.float32), (30, 1))
    b = P.bilateral_32f(ramp)
    assert np.allclose(b[:, 5:-5], ramp[:, 5:-5], atol=1e-5)           # a linear ramp stays linear inside
    g = P.sobel_mag(ramp)
    assert np.allclose(g[:, 1:-1], 8 * (ramp[0, 1] - ramp[0, 0]), rtol=1e-4)   # Sobel gain 8 on a ramp
    assert np.all(g[:, 0] == 0) and np.all(g[:, -1] == 0)                      # reflect-101 edges


def test_oracle_toon_edges_follow_depth():
    img, depth = scene()
    out = P.toon(img, P.depth_normalize(depth))
    q = (np.floor(img.astype(np.float32) / np.float32(255) * np.float32(5)) / np.float32(5) *
         np.float32(255)).astype(np.uint8)
    dark = np.all(out == 0, axis=2) & np.any(q > 0, axis=2)
    assert dark.any()
    H, W = depth.shape
    ys, xs = np.nonzero(dark)
    # every edge pixel lies within a few pixels of the box boundary
    assert np.all((np.abs(ys - H // 4) <= 6) | (np.abs(ys - 3 * H // 4) <= 6) |
                  (np.abs(xs - W // 3) <= 6) | (np.abs(xs - 2 * W // 3) <= 6))
    assert np.array_equal(out[~dark], q[~dark])


def test_numpy_cube_is_within_one_ulp_of_cube_rn():
    """The one host-dependent step of Fog: numpy's float32 `** 3.0` against cube_rn."""
    a = np.random.default_rng(0).random(1_000_000, dtype=np.float32)
    d = a ** np.float32(3.0)
    r = P.cube_rn(a)
    ulps = np.abs(d.view(np.int32).astype(np.int64) - r.view(np.int32))
    assert ulps.max() <= 1


@pytest.mark.parametrize("name", F9_CASES)
def test_oracle_fog_matches_reference_f9(name):
    """The oracle's Fog is the reference's, bit for bit (F9); with the kernel's rounded cube it
    differs only where numpy's float32 pow and the rounded cube disagree, by one count at most."""
    img, depth, start, ref, differs = f9_case(name)
    rn = P.fog(img, depth, fog_start=start, cube="rn")
    if depth is None:
        assert np.array_equal(rn, ref)
        return
    dn = np.array(depth if depth.ndim == 2 else depth[..., 0], np.float32)
    if dn.max() > 1.0:
        dn = dn / dn.max()
    a = np.clip(np.maximum(dn - np.float32(start), np.float32(0)) / np.float32(1.0 - start), 0, 1)
    host_pow_same = np.array_equal(a ** np.float32(3.0) != P.cube_rn(a), differs)
    if host_pow_same:   # this host's numpy pow rounds as the generating host's did
        assert np.array_equal(P.fog(img, depth, fog_start=start, cube="numpy"), ref)
    bad = np.any(rn != ref, axis=2)
    assert np.all(differs[bad])
    assert np.abs(rn.astype(int) - ref.astype(int)).max() <= 1


# --------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", F9_CASES)
def test_fog_matches_reference_f9(name):
    """The kernel's Fog against the reference's own outputs (F9): equal except where numpy's pow
    and the rounded cube disagree (stored per pixel in F9), and there within one count; equal to
    the oracle's rounded-cube form everywhere."""
    import nerfmi
    img, depth, start, ref, differs = f9_case(name)
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Fog"
    pp.params["fog_start"] = start
    got = pp.apply_effect(img, depth)
    assert np.array_equal(got, P.fog(img, depth, fog_start=start, cube="rn"))
    bad = np.any(got != ref, axis=2)
    if depth is None:
        assert not bad.any()
    else:
        assert np.all(differs[bad])
    assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1


@pytest.mark.gpu
def test_depth_normalize_matches_run_py():
    from nerfmi.post_processor import normalize_depth
    _, depth = scene()
    np.testing.assert_array_equal(normalize_depth(depth), P.depth_normalize(depth))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["normalized", "raw", "channels", "none"])
def test_fog_matches_oracle(mode):
    import nerfmi
    img, depth = scene(seed=3, H=400, W=400)
    d = {"normalized": P.depth_normalize(depth), "raw": depth, "none": None,
         "channels": np.repeat(P.depth_normalize(depth)[..., None], 4, axis=2)}[mode]
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Fog"
    got = pp.apply_effect(img, d)
    start = pp.params["fog_start"]
    assert np.array_equal(got, P.fog(img, d, fog_start=start, cube="rn"))        # bit-exact
    ref = P.fog(img, d, fog_start=start, cube="numpy")
    diff = np.any(got != ref, axis=2)
    if diff.any():   # only where numpy's SIMD pow and the rounded cube disagree
        dn = np.array(d if d.ndim == 2 else d[..., 0], np.float32)
        if dn.max() > 1.0:
            dn = dn / dn.max()
        a = np.clip(np.maximum(dn - np.float32(start), np.float32(0)) / np.float32(1.0 - start), 0, 1)
        assert np.all((a ** np.float32(3.0) != P.cube_rn(a))[diff])
        assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1
    # device tensors in, device tensor out
    t = pp.apply_effect(torch.from_numpy(img).cuda(), None if d is None else torch.from_numpy(np.ascontiguousarray(d)).cuda())
    assert t.is_cuda and np.array_equal(t.cpu().numpy(), got)


@pytest.mark.gpu
@pytest.mark.parametrize("const_depth", [False, True])
def test_frame_fog_is_the_cli_chain(const_depth):
    """nerf_frame_fog (run.py:233 truncation -> :248 normalisation -> Fog, one pass after the depth
    reduction) against the CLI's separate steps on the GPU and against the oracle chain, bit for
    bit.  rgb covers 0, 1 and every k/255 (the truncation boundaries)."""
    import nerfmi
    from nerfmi.post_processor import frame_fog, normalize_depth
    g = np.random.default_rng(7)
    H, W = 300, 400
    rgb = g.random((H, W, 3), dtype=np.float32)
    rgb.flat[:256] = np.arange(256, dtype=np.float32) / np.float32(255)
    rgb.flat[256:260] = [0.0, 1.0, np.nextafter(np.float32(1), np.float32(0)), 1e-8]
    _, depth = scene(seed=9, H=H, W=W)
    depth = depth + g.normal(0, 0.01, depth.shape).astype(np.float32)
    if const_depth:
        depth[:] = 3.25
    got = frame_fog(torch.from_numpy(rgb).cuda(), torch.from_numpy(depth).cuda()).cpu().numpy()
    img = (torch.from_numpy(rgb) * 255).numpy().astype(np.uint8)            # run.py:233
    assert np.array_equal(got, P.fog(img, P.depth_normalize(depth), fog_start=0.1, cube="rn"))
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Fog"
    assert np.array_equal(got, pp.apply_effect(img, normalize_depth(depth)))
    with pytest.raises(ValueError):
        frame_fog(torch.from_numpy(rgb).cuda(), torch.from_numpy(depth[:-1]).cuda())


@pytest.mark.gpu
@pytest.mark.parametrize("with_depth,levels", [(True, 5), (False, 5), (True, 4.5), (False, 7.25)])
def test_toon_matches_oracle(with_depth, levels):
    """Bit for bit, including a non-integer level count (the reference's editor stores
    float(value) in params, post_processor.py:67,72)."""
    import nerfmi
    img, depth = scene(seed=5, H=300, W=400)
    d = P.depth_normalize(depth) if with_depth else None
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Toon Shader"
    pp.params["toon_levels"] = levels
    got = pp.apply_effect(img, d)
    exp = P.toon(img, d, levels=levels, edge_strength=pp.params["toon_edge_strength"])
    assert np.array_equal(got, exp), float(np.mean(np.all(got == exp, axis=2)))


@pytest.mark.gpu
def test_effect_errors():
    import nerfmi
    pp = nerfmi.PostProcessor()
    img, depth = scene()
    pp.current_effect = "Sepia"
    with pytest.raises(NotImplementedError):
        pp.apply_effect(img, depth)
    pp.current_effect = "Fog"
    with pytest.raises(ValueError):
        pp.apply_effect(img[:, :, :2].copy(), depth)
    with pytest.raises(ValueError):
        pp.apply_effect(img, depth[:-1])
    pp.current_effect = "Original"
    assert pp.apply_effect(img, depth) is img
