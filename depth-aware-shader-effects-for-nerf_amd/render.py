"""volume_render / render_rays (src/render.py of the reference), one C-ABI call per invocation.

``volume_render(model, rays_o, rays_d, near, far, n_samples, n_importance,
appearance_embedding=None, background_color=None, perturb=True)`` has the reference's
signature and return value ``(rgb_map (...,3), depth_map (...,1), extras)`` with
``extras = {'weights': (B,N,1), 'z_vals': (B,N)}`` (render.py:5-97).  By default it keeps
the reference's semantics exactly, including ignoring ``n_importance`` (render.py:83-86)
and ``background_color``.  Keyword-only extras:
  hierarchical=True   H1 fine pass: resample n_importance samples from the coarse weights
                      and composite over all N+Nf merged samples; extras then also hold the
                      coarse maps/weights/z ('rgb_map_coarse', ...).
  t_rand, u_rand      explicit uniforms for the stratified jitter (B,N) and the inverse-CDF
                      draw (B,Nf) — the reference's torch.rand draws (ray_utils.py:80,119).
  seed                key of the in-kernel RNG when no uniforms are given (drawn from the
                      torch CPU generator by default).
  ray_offset          global index of the first ray: the in-kernel draws of ray r are those of
                      ray ray_offset + r of one big batch, so ray shards rendered separately equal
                      the batch rendered at once, bit for bit (frames.py; include/nerfmi.h).
  timing              optional list; when given, the path runs stage by stage and appends
                      (start, end, samples) per fused-MLP launch, the events recorded around
                      the launch on this stream (bench.py's roofline leg).
  staged, reuse_coarse  staged=True runs the per-stage entry points instead of the single
                      nerf_render_rays call; reuse_coarse=False (staged only) re-evaluates the
                      coarse samples in the fine pass — bit-identical, for the tests.
``render_rays`` is the same function (the north-star name).

With gradients enabled and a trainable model (or an appearance embedding that requires grad),
the reference-compat call (coarse; hierarchical, staged and timing unset) runs the training
kernels instead (autograd.py): rgb_map and depth_map carry a grad_fn whose backward is the
composite backward + MLP data-gradient chain + weight-gradient reductions of csrc/train.hip, as
the reference's training loop needs (src/train.py:77-92).  The H1 hierarchical pass has no
reference training semantics (render.py:83-86 is a stub): with gradients enabled and a trainable
model it raises (RuntimeError naming hierarchical=True) instead of silently returning no graph.
"""
import torch

from . import _lib
from .models import STATE_KEYS, app_rows, pack_params, run_mlp, state_tensors, uses_appearance
from .ray_utils import draw_seed, linspace_table, rng_key_at

_IMPORTANCE_KEY = 0x5DEECE66D     # the inverse-CDF stream's key: seed ^ this (include/nerfmi.h)


def packed_for(model):
    """Packed weights of a nerfmi.NeRF, or of any module with the reference's state_dict keys
    (e.g. the reference's own NeRF after load_state_dict)."""
    if hasattr(model, "packed_weights"):
        return model.packed_weights()
    dev = _lib.device()
    sd = model.state_dict()
    key = (dev,) + tuple((sd[k].data_ptr(), sd[k]._version) for k in STATE_KEYS if k in sd)
    hit = model.__dict__.get("_nerfmi_packed")          # cached on the module: lives and dies with it
    if hit is None or hit[0] != key:
        hit = model.__dict__["_nerfmi_packed"] = (key, pack_params(state_tensors(sd, dev), dev))
    return hit[1]


def volume_render(model, rays_o, rays_d, near, far, n_samples, n_importance, appearance_embedding=None,
                  background_color=None, perturb=True, *, hierarchical=False, t_rand=None, u_rand=None,
                  seed=None, ray_offset=0, timing=None, staged=False, reuse_coarse=True):
    from . import autograd
    if autograd.needs_grad(model, appearance_embedding if uses_appearance(model) else None, rays_o, rays_d):
        if hierarchical or staged or timing is not None:
            what = "hierarchical=True" if hierarchical else ("staged=True" if staged else "timing=")
            raise RuntimeError(
                f"nerfmi.volume_render({what}) has no differentiable path: the reference's fine pass is a stub "
                f"with no training semantics (src/render.py:83-86) and the staged/timed paths are inference "
                f"instrumentation.  Render under torch.no_grad() (as the reference's run.py:217 does) or with "
                f"parameters that do not require grad; the coarse call (hierarchical=False) is differentiable.")
        return autograd.volume_render_grad(model, rays_o, rays_d, near, far, n_samples, appearance_embedding,
                                           perturb, t_rand=t_rand, seed=seed, ray_offset=ray_offset)
    dev = _lib.device()
    lib = _lib.load()
    orig_shape = rays_o.shape
    o = rays_o.reshape(-1, 3).to(dev, torch.float32).contiguous()
    d = rays_d.reshape(-1, 3).to(dev, torch.float32).contiguous()
    B = o.shape[0]
    N = int(n_samples)
    Nf = int(n_importance) if hierarchical else 0
    T = N + Nf
    packed = packed_for(model)
    app, rows = app_rows(appearance_embedding if uses_appearance(model) else None, B, dev)
    tr = t_rand.reshape(B, N).to(dev, torch.float32).contiguous() if (perturb and t_rand is not None) else None
    ur = u_rand.reshape(B, Nf).to(dev, torch.float32).contiguous() if (Nf and u_rand is not None) else None
    if seed is None and ((perturb and tr is None) or (Nf and ur is None)):
        seed = draw_seed()
    t_vals = linspace_table(N, dev)
    u_lin = linspace_table(Nf, dev, drop_last=True) if Nf else None

    rgb_map = torch.empty(B, 3, device=dev)
    depth_map = torch.empty(B, 1, device=dev)
    weights = torch.empty(B, T, 1, device=dev)
    z_vals = torch.empty(B, T, device=dev)
    extras = {}
    if Nf:
        crgb = torch.empty(B, 3, device=dev)
        cdepth = torch.empty(B, 1, device=dev)
    if timing is None and not staged:
        ws = torch.empty(lib.nerf_render_workspace_bytes(B, N, Nf), dtype=torch.uint8, device=dev)
        _lib.check(lib.nerf_render_rays(
            _lib.ptr(packed), _lib.ptr(o), _lib.ptr(d), B, float(near), float(far), N, Nf, _lib.ptr(t_vals),
            _lib.ptr(u_lin), int(bool(perturb)), _lib.ptr(tr), _lib.ptr(ur), seed or 0, int(ray_offset),
            _lib.ptr(app), rows,
            _lib.ptr(rgb_map), _lib.ptr(depth_map), _lib.ptr(weights), _lib.ptr(z_vals),
            _lib.ptr(crgb) if Nf else None, _lib.ptr(cdepth) if Nf else None, _lib.ptr(ws), ws.numel(),
            _lib.stream()), "nerf_render_rays")
        if Nf:
            cw, cz = None, None
    else:
        cw, cz = _staged(lib, packed, o, d, B, near, far, N, Nf, t_vals, u_lin, perturb, tr, ur, seed or 0,
                         int(ray_offset), app, rows, rgb_map, depth_map, weights, z_vals, crgb if Nf else None,
                         cdepth if Nf else None, timing, reuse_coarse)
    out = rays_o.device
    if T == 1:   # the reference's per-sample tensors are empty at one sample (render.py:56-58)
        weights = weights[:, :0]
    extras["weights"] = weights.to(out)
    extras["z_vals"] = z_vals.to(out)
    if Nf:
        extras["rgb_map_coarse"] = crgb.reshape(*orig_shape[:-1], 3).to(out)
        extras["depth_map_coarse"] = cdepth.reshape(*orig_shape[:-1], 1).to(out)
        if cw is not None:
            extras["weights_coarse"] = cw.unsqueeze(-1).to(out)
            extras["z_vals_coarse"] = cz.to(out)
    return (rgb_map.reshape(*orig_shape[:-1], 3).to(out), depth_map.reshape(*orig_shape[:-1], 1).to(out), extras)


def _staged(lib, packed, o, d, B, near, far, N, Nf, t_vals, u_lin, perturb, tr, ur, seed, ray0, app, rows, rgb_map,
            depth_map, weights, z_out, crgb, cdepth, timing, reuse_coarse=True):
    """The kernel sequence of nerf_render_rays, issued stage by stage through the per-stage entry
    points so every fused-MLP launch can be bracketed by events on this stream.  With
    reuse_coarse=False the fine pass re-evaluates all N+Nf merged samples instead (the reference
    semantics spelled out; bit-identical results, used by the tests)."""
    dev = o.device
    s = _lib.stream()
    P = _lib.ptr
    dn = torch.empty_like(d)
    _lib.check(lib.nerf_normalize_dirs(P(d), B, P(dn), s), "nerf_normalize_dirs")
    z = torch.empty(B, N, device=dev)
    _lib.check(lib.nerf_sample_stratified(P(o), P(dn), B, float(near), float(far), N, P(t_vals), int(bool(perturb)),
                                          P(tr), rng_key_at(seed, ray0 * N), P(z), None, s), "nerf_sample_stratified")
    feat = torch.empty(B, 256, device=dev)
    _lib.check(lib.nerf_ray_features(P(packed), P(dn), B, P(app), rows, P(feat), s), "nerf_ray_features")
    T = N + Nf

    def mlp(zz, n, rgb, sigma, slot=None):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        _lib.check(lib.nerf_mlp_forward(P(packed), P(o), P(dn), P(zz), B, n, P(feat), P(rgb), P(sigma), P(slot),
                                        T, s), "nerf_mlp_forward")
        ev[1].record()
        if timing is not None:
            timing.append((ev[0], ev[1], B * n))

    rgb_c = torch.empty(B * N, 3, device=dev)
    sigma_c = torch.empty(B * N, device=dev)
    mlp(z, N, rgb_c, sigma_c)
    if not Nf:
        _lib.check(lib.nerf_composite(P(rgb_c), P(sigma_c), P(z), B, N, P(rgb_map), P(depth_map), P(weights), s),
                   "nerf_composite")
        z_out.copy_(z)
        return None, None
    wc = torch.empty(B, N, device=dev)
    _lib.check(lib.nerf_composite(P(rgb_c), P(sigma_c), P(z), B, N, P(crgb), P(cdepth), P(wc), s), "nerf_composite")
    rgb_all = torch.empty(B * T, 3, device=dev)
    sigma_all = torch.empty(B * T, device=dev)
    key = rng_key_at(seed ^ _IMPORTANCE_KEY, ray0 * Nf)
    if reuse_coarse:
        z_fine = torch.empty(B, Nf, device=dev)
        slot = torch.empty(B, Nf, dtype=torch.int32, device=dev)
        _lib.check(lib.nerf_sample_importance_merge(P(z), P(wc), P(rgb_c), P(sigma_c), B, N, Nf, P(u_lin), P(ur), key,
                                                    P(z_out), P(rgb_all), P(sigma_all), P(z_fine), P(slot), s),
                   "nerf_sample_importance_merge")
        mlp(z_fine, Nf, rgb_all, sigma_all, slot)
    else:
        _lib.check(lib.nerf_sample_importance(P(o), P(dn), P(z), P(wc), B, N, Nf, P(u_lin), P(ur), key, P(z_out),
                                              None, s), "nerf_sample_importance")
        mlp(z_out, T, rgb_all, sigma_all)
    _lib.check(lib.nerf_composite(P(rgb_all), P(sigma_all), P(z_out), B, T, P(rgb_map), P(depth_map), P(weights),
                                  s), "nerf_composite")
    return wc, z


render_rays = volume_render
