"""Depth-aware post effects: nerfmi.PostProcessor's GPU kernels
(csrc/effects.hip) against oracle/post_oracle.py, and the oracle's own properties on the CPU.

Parity unpinned against the reference itself: src/post_processor.py imports cv2 and tkinter,
which are absent, so it cannot run here.  The oracle restates Fog and the numpy steps of Toon
operation for operation and the cv2 steps from OpenCV 4's algorithms (oracle/post_oracle.py).
Tolerances: the outputs are uint8 after truncation; Fog's x**3 is powf on both sides (glibc vs
the device library, both ~1 ulp), so a value may land one count apart at a truncation boundary:
at most 1 count on at most 0.5% of values.  Toon's edge mask must agree on >= 99.9% of pixels
(the bilateral filter's float sums are compared at 1e-6 relative).
"""
import numpy as np
import pytest
import torch

from oracle import post_oracle as P


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


# --------------------------------------------------------------------------------- GPU
def _close_u8(got, exp, frac=0.005):
    d = np.abs(got.astype(np.int16) - exp.astype(np.int16))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() <= frac, (d > 0).mean()


@pytest.mark.gpu
def test_depth_normalize_matches_run_py():
    from nerfmi.post_processor import normalize_depth
    _, depth = scene()
    np.testing.assert_array_equal(normalize_depth(depth), P.depth_normalize(depth))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["normalized", "raw", "channels", "none"])
def test_fog_matches_oracle(mode):
    import nerfmi
    img, depth = scene(seed=3)
    d = {"normalized": P.depth_normalize(depth), "raw": depth, "none": None,
         "channels": np.repeat(P.depth_normalize(depth)[..., None], 4, axis=2)}[mode]
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Fog"
    got = pp.apply_effect(img, d)
    _close_u8(got, P.fog(img, d, fog_start=pp.params["fog_start"]))
    # device tensors in, device tensor out
    t = pp.apply_effect(torch.from_numpy(img).cuda(), None if d is None else torch.from_numpy(np.ascontiguousarray(d)).cuda())
    assert t.is_cuda and np.array_equal(t.cpu().numpy(), got)


@pytest.mark.gpu
@pytest.mark.parametrize("with_depth", [True, False])
def test_toon_matches_oracle(with_depth):
    import nerfmi
    img, depth = scene(seed=5)
    d = P.depth_normalize(depth) if with_depth else None
    pp = nerfmi.PostProcessor()
    pp.current_effect = "Toon Shader"
    got = pp.apply_effect(img, d)
    exp = P.toon(img, d, levels=pp.params["toon_levels"], edge_strength=pp.params["toon_edge_strength"])
    same = np.all(got == exp, axis=2)
    assert same.mean() >= 0.999, same.mean()


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
