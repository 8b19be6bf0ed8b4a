"""CPU oracle for the depth-aware post effects — TEST INFRASTRUCTURE ONLY.

The checker for csrc/effects.hip (nerfmi.PostProcessor): a numpy restatement of the reference's
`PostProcessor._effect_fog` (src/post_processor.py:451-493), `_effect_toon` (:64-117) and the depth
normalisation of run.py (run.py:248).  Only tests/ import it.

Pinning.  The reference module imports cv2 and tkinter at the top (post_processor.py:2-4), neither
of which is installed here, so it cannot be imported as a whole.  Its Fog method is numpy alone:
tests/golden/make_post_golden.py compiles that one method from the module's source and records its
outputs as fixture F9, and `fog(cube="numpy")` equals F9 bit for bit (tests/test_post_effects.py).
Toon is **parity unpinned**: its quantisation/combination steps are numpy expressions restated
here operation for operation (float32 arrays, Python scalars taken as float32 by numpy's
weak-scalar rule, astype(uint8) truncating after np.clip), and its cv2 calls (cvtColor RGB2GRAY,
bilateralFilter, Sobel, Laplacian, dilate) are restated from OpenCV 4's published algorithms
(fixed-point gray, bilateralFilter_32f's 4096-bin colour LUT, separable Sobel, reflect-101
borders, dilation ignoring the border); cv2 itself is not available to pin them.
"""
import math

import numpy as np

F32 = np.float32


def depth_normalize(depth):
    """run.py:248: (d - min) / (max - min + 1e-6) on a float32 depth image."""
    d = np.asarray(depth, F32)
    return (d - d.min()) / (d.max() - d.min() + F32(1e-6))


def cube_rn(a):
    """a**3 rounded once to float32 (a*a exact in float64, the second product rounded to float64,
    then to float32): the cube csrc/effects.hip computes."""
    d = np.asarray(a, np.float64)
    return ((d * d) * d).astype(F32)


def fog(image, depth=None, fog_start=0.1, cube="numpy"):
    """post_processor.py:451-493.  The fog colour is pure white (:455-459); density and the
    fog colour parameters are read but unused by the reference.  cube="numpy" is the reference's
    `adjusted ** 3.0` (numpy's float32 SIMD pow: SVML on AVX-512 hosts, within 1 ulp of the
    correctly rounded cube and host-dependent); cube="rn" is cube_rn, the kernel's."""
    fog_color = np.array([255, 255, 255], dtype=F32)
    if depth is None:
        result = image.astype(F32) * F32(0.05) + fog_color * F32(0.95)
        return np.clip(result, 0, 255).astype(np.uint8)
    depth_norm = np.array(depth, dtype=F32, copy=True)
    if depth_norm.ndim > 2:
        depth_norm = depth_norm[:, :, 0]
    if depth_norm.max() > 1.0:
        depth_norm = depth_norm / depth_norm.max()
    adjusted = np.maximum(depth_norm - F32(fog_start), F32(0.0)) / F32(1.0 - fog_start)
    adjusted = np.clip(adjusted, F32(0.0), F32(1.0))
    adjusted = adjusted ** F32(3.0) if cube == "numpy" else cube_rn(adjusted)
    adjusted = adjusted * F32(0.3)
    f3 = np.stack([adjusted] * 3, axis=2)
    result = image.astype(F32) * f3 + fog_color * (F32(1.0) - f3)
    return np.clip(result, 0, 255).astype(np.uint8)


def _reflect101(i, n):
    if n == 1:
        return np.zeros_like(i)
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


def _shift(a, dy, dx):
    """a[reflect101(y+dy), reflect101(x+dx)] for every (y, x)."""
    H, W = a.shape
    ys = _reflect101(np.arange(H) + dy, H)
    xs = _reflect101(np.arange(W) + dx, W)
    return a[ys][:, xs]


def bilateral_32f(src, d=9, sigma_color=75.0, sigma_space=75.0):
    """cv2.bilateralFilter on one float32 channel (OpenCV 4 bilateralFilter_32f)."""
    src = np.asarray(src, F32)
    radius = max(d // 2, 1)
    mn, mx = float(src.min()), float(src.max())
    if abs(mn - mx) < np.finfo(np.float32).eps:
        return src.copy()
    gcc = -0.5 / (sigma_color * sigma_color)
    gsc = -0.5 / (sigma_space * sigma_space)
    nbins = 1 << 12
    length = F32(mx - mn)
    scale_index = F32(F32(nbins) / length)
    lut = np.empty(nbins + 2, F32)
    for i in range(nbins + 2):
        v = float(F32(F32(i) / scale_index))
        lut[i] = F32(math.exp(v * v * gcc))
    sum_ = np.zeros_like(src)
    wsum = np.zeros_like(src)
    for i in range(-radius, radius + 1):
        for j in range(-radius, radius + 1):
            r = math.sqrt(i * i + j * j)
            if r > radius or (i == 0 and j == 0):
                continue
            sw = F32(math.exp(r * r * gsc))
            val = _shift(src, i, j)
            alpha = (np.abs(val - src) * scale_index).astype(F32)
            idx = np.floor(alpha).astype(np.int64)
            alpha = (alpha - idx.astype(F32)).astype(F32)
            w = (sw * (lut[idx] + alpha * (lut[idx + 1] - lut[idx]))).astype(F32)
            wsum = (wsum + w).astype(F32)
            sum_ = (sum_ + val * w).astype(F32)
    return ((sum_ + src) / (wsum + F32(1.0))).astype(F32)


def sobel_mag(f):
    """sqrt(Sobel_x^2 + Sobel_y^2) (cv2.Sobel ksize 3, CV_32F, separable, reflect-101)."""
    f = np.asarray(f, F32)
    r = {k: _shift(f, k, 1) - _shift(f, k, -1) for k in (-1, 0, 1)}
    gx = r[0] * F32(2.0) + (r[-1] + r[1])
    h = {k: _shift(f, k, 0) * F32(2.0) + (_shift(f, k, -1) + _shift(f, k, 1)) for k in (-1, 1)}
    gy = h[1] - h[-1]
    return np.sqrt(gx * gx + gy * gy)


def gray_u8(image):
    """cv2.cvtColor(RGB2GRAY) on uint8: 14-bit fixed point 0.299/0.587/0.114, rounded."""
    im = image.astype(np.int64)
    return ((im[..., 0] * 4899 + im[..., 1] * 9617 + im[..., 2] * 1868 + (1 << 13)) >> 14).astype(F32)


def laplacian_abs(gray):
    """|cv2.Laplacian(gray, CV_32F)| (ksize 1: [0 1 0; 1 -4 1; 0 1 0], reflect-101)."""
    g = np.asarray(gray, F32)
    lap = _shift(g, -1, 0) + _shift(g, 0, -1) + _shift(g, 0, 1) + _shift(g, 1, 0) - F32(4.0) * g
    return np.abs(lap)


def dilate3(mask):
    """cv2.dilate with a 3x3 box, one iteration, pixels outside the image ignored."""
    m = np.asarray(mask, bool)
    H, W = m.shape
    p = np.zeros((H + 2, W + 2), bool)
    p[1:-1, 1:-1] = m
    out = np.zeros_like(m)
    for dy in range(3):
        for dx in range(3):
            out |= p[dy:dy + H, dx:dx + W]
    return out


def toon(image, depth=None, levels=5, edge_strength=1.0):
    """post_processor.py:64-117 (`levels` as the reference uses it: a numpy weak scalar, so
    float32(levels), integer or not)."""
    img_float = image.astype(F32)
    img_q = np.floor(img_float / F32(255.0) * F32(levels)) / F32(levels) * F32(255.0)
    if depth is not None:
        depth_norm = np.array(depth, dtype=F32, copy=True)
        if depth_norm.max() > 1.0:
            depth_norm = depth_norm / depth_norm.max()
        filt = bilateral_32f(depth_norm, 9, 75, 75)
        grad = sobel_mag(filt)
        if grad.max() > 0:
            grad = grad / grad.max()
        edges = dilate3(grad > F32(0.05)).astype(F32)
    else:
        lap = laplacian_abs(gray_u8(image))
        if lap.max() > 0:
            lap = lap / lap.max()
        edges = (lap > F32(0.1)).astype(F32)
    e3 = np.stack([edges] * 3, axis=2)
    result = img_q * (F32(1.0) - F32(edge_strength) * e3)
    return np.clip(result, 0, 255).astype(np.uint8)
