"""Ray generation and sampling (src/ray_utils.py of the reference), computed by libnerfmi.so.

Same names, argument meaning and return shapes as the reference:
  get_rays(height, width, focal_length, c2w)                 ray_utils.py:4-50
  sample_stratified(rays_o, rays_d, near, far, n_samples, perturb=True)   :52-88
  sample_importance(rays_o, rays_d, z_vals, weights, n_importance)        :90-149 (H1)
Keyword-only extras: ``t_rand`` / ``u_rand`` take the uniforms explicitly (the reference
draws them with torch.rand from the CPU generator, :80 and :119), ``seed`` keys the
in-kernel counter RNG when no uniforms are given (by default a seed is drawn from the
torch CPU generator, so torch.manual_seed makes runs repeatable).
Results come back on the device of the inputs; the arithmetic always runs on the GPU.
"""
import ctypes

import torch

from . import _lib

_TABLES = {}


def linspace_table(n, dev, drop_last=False):
    """torch.linspace(0, 1, n) (ray_utils.py:69) or linspace(0, 1, n+1)[:-1] (:115) as a cached
    device table: the CPU linspace is what the reference evaluates, so its exact values are used."""
    key = (n, drop_last, dev)
    if key not in _TABLES:
        t = torch.linspace(0., 1., n + 1)[:-1] if drop_last else torch.linspace(0., 1., n)
        _TABLES[key] = t.to(dev).contiguous()
    return _TABLES[key]


def draw_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


_GOLDEN64 = 0x9E3779B97F4A7C15
_MASK64 = (1 << 64) - 1


def rng_key_at(seed, first):
    """Key of the in-kernel uniform stream shifted to index `first`: u(rng_key_at(s, f), i) ==
    u(s, f + i) (csrc/common.h rng_key_at; include/nerfmi.h nerf_rng_uniforms)."""
    return (int(seed) + _GOLDEN64 * int(first)) & _MASK64


def get_rays(height, width, focal_length, c2w, *, rows=None):
    """origins (H,W,3) — a 0-stride expand of c2w[:3,3] as in the reference (:48) — and unit
    directions (H,W,3) on c2w's device.  rows=(row0, nrows) generates only those image rows
    ((nrows,W,3) outputs; the frame sharding of frames.py)."""
    if c2w.shape[-1] != 4 or c2w.dim() != 2 or c2w.shape[0] not in (3, 4):
        raise ValueError(f"get_rays: c2w must be (3,4) or (4,4), got {tuple(c2w.shape)}")
    dev = _lib.device()
    row0, nrows = (0, height) if rows is None else (int(rows[0]), int(rows[1]))
    m = c2w[:3, :4].detach().to("cpu", torch.float32).contiguous()
    host = (ctypes.c_float * 12)(*m.flatten().tolist())
    d = torch.empty(nrows, width, 3, device=dev)
    _lib.check(_lib.load().nerf_get_rays(height, width, float(focal_length), host, row0, nrows, None, _lib.ptr(d),
                                         _lib.stream()), "nerf_get_rays")
    d = d.to(c2w.device)
    return c2w[..., :3, 3].to(torch.float32).expand(d.shape), d


def rays_on_device(height, width, focal_length, c2w_host, rows, dev):
    """Device (o, d), each (nrows*W, 3), of image rows rows=(row0, nrows) from a host c2w
    (list/array of 12 floats or a CPU (3,4)/(4,4) tensor): no device-to-host copy of the pose, so a
    shard loop issues no synchronisation (frames.py)."""
    m = torch.as_tensor(c2w_host, dtype=torch.float32).reshape(-1, 4)[:3].contiguous()
    host = (ctypes.c_float * 12)(*m.flatten().tolist())
    row0, nrows = int(rows[0]), int(rows[1])
    d = torch.empty(nrows * width, 3, device=dev)
    _lib.check(_lib.load().nerf_get_rays(height, width, float(focal_length), host, row0, nrows, None, _lib.ptr(d),
                                         _lib.stream()), "nerf_get_rays")
    o = m[:, 3].to(dev, non_blocking=True).expand(d.shape)
    return o, d


def sample_stratified(rays_o, rays_d, near, far, n_samples, perturb=True, *, t_rand=None, seed=None):
    """z_vals (..., N) and pts (..., N, 3)."""
    dev = _lib.device()
    lead = rays_o.shape[:-1]
    o = rays_o.reshape(-1, 3).to(dev, torch.float32).contiguous()
    d = rays_d.reshape(-1, 3).to(dev, torch.float32).contiguous()
    B = o.shape[0]
    z = torch.empty(B, n_samples, device=dev)
    pts = torch.empty(B, n_samples, 3, device=dev)
    tr = None
    if perturb and t_rand is not None:
        tr = t_rand.reshape(B, n_samples).to(dev, torch.float32).contiguous()
    if perturb and tr is None and seed is None:
        seed = draw_seed()
    _lib.check(_lib.load().nerf_sample_stratified(
        _lib.ptr(o), _lib.ptr(d), B, float(near), float(far), n_samples, _lib.ptr(linspace_table(n_samples, dev)),
        int(bool(perturb)), _lib.ptr(tr), seed or 0, _lib.ptr(z), _lib.ptr(pts), _lib.stream()),
        "nerf_sample_stratified")
    out = rays_o.device
    return z.reshape(*lead, n_samples).to(out), pts.reshape(*lead, n_samples, 3).to(out)


def sample_importance(rays_o, rays_d, z_vals, weights, n_importance, *, u_rand=None, seed=None):
    """H1 inverse-CDF resampling: z_vals_combined (..., N+Nf) sorted and pts_combined (..., N+Nf, 3).
    Identical to the reference wherever the reference does not raise."""
    dev = _lib.device()
    lead = rays_o.shape[:-1]
    N = z_vals.shape[-1]
    if weights.dim() == z_vals.dim() + 1 and weights.shape[-1] == 1:
        weights = weights[..., 0]
    o = rays_o.reshape(-1, 3).to(dev, torch.float32).contiguous()
    d = rays_d.reshape(-1, 3).to(dev, torch.float32).contiguous()
    B = o.shape[0]
    z = z_vals.reshape(B, N).to(dev, torch.float32).contiguous()
    w = weights.reshape(B, N).to(dev, torch.float32).contiguous()
    ur = None
    if u_rand is not None:
        ur = u_rand.reshape(B, n_importance).to(dev, torch.float32).contiguous()
    elif seed is None:
        seed = draw_seed()
    T = N + n_importance
    z_all = torch.empty(B, T, device=dev)
    pts = torch.empty(B, T, 3, device=dev)
    _lib.check(_lib.load().nerf_sample_importance(
        _lib.ptr(o), _lib.ptr(d), _lib.ptr(z), _lib.ptr(w), B, N, n_importance,
        _lib.ptr(linspace_table(n_importance, dev, drop_last=True)), _lib.ptr(ur), seed or 0, _lib.ptr(z_all),
        _lib.ptr(pts), _lib.stream()), "nerf_sample_importance")
    out = rays_o.device
    return z_all.reshape(*lead, T).to(out), pts.reshape(*lead, T, 3).to(out)
