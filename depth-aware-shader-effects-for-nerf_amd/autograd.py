"""Autograd over the HIP training kernels: the differentiable render path.

The reference trains by rendering with gradients enabled and calling ``loss.backward()``
(src/train.py:77-92); its run.py train mode also calls ``model(x, d, app)`` with gradients
enabled (run.py:338-345).  Here both run the training kernels of csrc/train.hip through the C ABI
(include/nerfmi_train.h), wrapped in two ``torch.autograd.Function``s:

  _RenderFn   volume_render (render.py:5-97, coarse; n_importance ignored as in :83-86)
              forward:  normalize -> stratified -> ray features -> fused PE->MLP forward that saves
                        every activation (+ ReLU mask rows under f16x3) -> composite (weights out)
              backward: nerf_composite_backward_grad (any upstream gradient of rgb_map and
                        depth_map) -> nerf_mlp_backward (data-gradient chain on MFMA) ->
                        nerf_param_grads (every weight/bias gradient as an MFMA reduction over the
                        samples, and the appearance rows' gradient)
  _MLPFn      NeRF.forward (models.py:105-162) on sample points: the same forward with saves (one
              "ray" per point, z = 0) and the same backward from d rgb, d sigma.

Gradients flow to every parameter of the model (state_dict keys of models.py:58-103) and to the
appearance embedding (an nn.Parameter row of the dataset's table in the reference's loop); they are
accumulated into ``.grad`` by autograd as usual, so ``torch.optim.Adam`` over ``model.parameters()``
plus the table steps exactly as in the reference.  Gradients with respect to ray origins,
directions or sample positions are not part of the reference's training and are refused loudly.
``extras['weights']`` and ``extras['z_vals']`` are returned without a gradient (marked
non-differentiable: a loss built on them alone raises at backward instead of returning zeros).
"""
import ctypes

import torch

from . import _lib
from .models import APP_KEYS, STATE_KEYS, app_rows, state_tensors, uses_appearance
from .ray_utils import draw_seed, linspace_table, rng_key_at

# parameters that only the colour branch reads (models.py:141-160): no gradient when the loss does
# not depend on rgb, as autograd leaves them (None, so torch.optim skips them)
_COLOUR_KEYS = ("dir_linear.weight", "dir_linear.bias", "appearance_projection.weight",
                "appearance_projection.bias", "rgb_linear.weight", "rgb_linear.bias")
_SIGMA_KEYS = ("density_head.weight", "density_head.bias")


def model_params(model):
    """(keys, parameters) of the model in STATE_KEYS order (22 without appearance_projection)."""
    named = dict(model.named_parameters())
    keys = [k for k in STATE_KEYS if k in named]
    return keys, [named[k] for k in keys]


def needs_grad(model, app, *inputs):
    """True when this call must be differentiable: gradients enabled and a trainable parameter
    (or the appearance embedding) requires grad."""
    if not torch.is_grad_enabled():
        return False
    params = [p for p in model.parameters() if p.requires_grad]
    trainable = bool(params) or (app is not None and app.requires_grad)
    if trainable and any(isinstance(t, torch.Tensor) and t.requires_grad for t in inputs):
        raise NotImplementedError("nerfmi: gradients with respect to ray origins / directions / sample positions "
                                  "are not computed (the reference trains the MLP and the appearance table only, "
                                  "src/train.py:36-39); detach them")
    return trainable


def packed_pair(model):
    """(packed, packedT): the forward layout (render.packed_for) and the transposed weight fragments
    the data-gradient chain reads, both re-packed when a parameter changes.  packedT is cached on the
    module itself (it lives and dies with the model; the key holds each parameter's address and
    version counter, so an in-place update or a new tensor re-packs)."""
    from .render import packed_for
    packed = packed_for(model)
    dev = packed.device
    sd = model.state_dict()
    key = (dev,) + tuple((sd[k].data_ptr(), sd[k]._version) for k in STATE_KEYS if k in sd)
    hit = model.__dict__.get("_nerfmi_packedT")
    if hit is None or hit[0] != key:
        lib = _lib.load()
        # (copies of host or non-fp32 parameters are freed after the pack is queued: the caching
        # allocator reuses their memory only for work queued after it on this stream)
        ts = [t.detach().to(dev, torch.float32).contiguous() for t in state_tensors(sd, dev)]
        arr = (ctypes.c_void_p * 24)(*[t.data_ptr() for t in ts])
        packedT = torch.empty(lib.nerf_packed_transposed_floats(), device=dev)
        _lib.check(lib.nerf_pack_weights_transposed(arr, _lib.ptr(packedT), _lib.stream()),
                   "nerf_pack_weights_transposed")
        hit = model.__dict__["_nerfmi_packedT"] = (key, packedT)
    return packed, hit[1]


def _grad_buffers(dev):
    """24 gradient tensors in STATE_KEYS order (one flat buffer) and their pointer array."""
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 3 + [(256, 319), (256,)] + [(256, 256), (256,)] * 3 + \
             [(1, 256), (1,), (128, 283), (128,), (128, 32), (128,), (3, 128), (3,)]
    sizes = [int(torch.Size(s).numel()) for s in shapes]
    flat = torch.empty(sum(sizes), device=dev)
    views, at = [], 0
    for s, n in zip(shapes, sizes):
        views.append(flat[at:at + n].view(s))
        at += n
    return views, (ctypes.c_void_p * 24)(*[v.data_ptr() for v in views])


def _param_grads(keys, params, app, rows, save, grad, M, N, packed, need_app, unused=()):
    """nerf_param_grads into fresh buffers: the gradients of `params` (in order) and of the appearance
    rows (rows x 32, or None).  Keys in `unused` (off the loss's path) get None."""
    lib = _lib.load()
    dev = save.device
    views, ptrs = _grad_buffers(dev)
    dapp = torch.empty(max(rows, 1), 32, device=dev) if (rows and need_app) else None
    ws = torch.empty(lib.nerf_param_grads_workspace_bytes(M), dtype=torch.uint8, device=dev)
    _lib.check(lib.nerf_param_grads(_lib.ptr(save), _lib.ptr(grad), M, N, _lib.ptr(app), rows, _lib.ptr(packed),
                                    ptrs, _lib.ptr(dapp), _lib.ptr(ws), ws.numel(), _lib.stream()),
               "nerf_param_grads")
    by_key = dict(zip(STATE_KEYS, views))
    out = []
    for k, p in zip(keys, params):
        if (k in APP_KEYS and rows == 0) or k in unused:   # not on the path (models.py:146): no gradient
            out.append(None)
            continue
        g = by_key[k]
        out.append(g if p.device == dev else g.to(p.device))
    return out, dapp


def _mlp_backward(packed, packedT, save, masks, sigma, rgb, dsigma, drgb, M):
    lib = _lib.load()
    grad = torch.empty(_lib.tile_rows(M), _lib.GRAD_ROW, device=save.device)   # tile-major rows
    _lib.check(lib.nerf_mlp_backward(_lib.ptr(packed), _lib.ptr(packedT), _lib.ptr(save), _lib.ptr(masks),
                                     _lib.ptr(sigma), _lib.ptr(rgb), _lib.ptr(dsigma), _lib.ptr(drgb), M,
                                     _lib.ptr(grad), _lib.stream()), "nerf_mlp_backward")
    return grad


def _app_grad(dapp, app):
    if dapp is None or app is None:
        return None
    return dapp.reshape(app.shape).to(app.device)


class _RenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, app, *params):
        lib, s, P = _lib.load(), _lib.stream(), _lib.ptr
        o, d, B, N = spec["o"], spec["d"], spec["B"], spec["N"]
        packed, packedT = spec["packed"], spec["packedT"]
        appd, rows = spec["app"], spec["rows"]
        dev = o.device
        M = B * N
        dn = torch.empty(B, 3, device=dev)
        z = torch.empty(B, N, device=dev)
        feat, encd = torch.empty(B, 256, device=dev), torch.empty(B, 32, device=dev)
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
        save = torch.empty(_lib.tile_rows(M), _lib.SAVE_ROW, device=dev)   # tile-major rows
        arith = _lib.get_mlp_arith()
        masks = torch.empty(M, _lib.MASK_ROW, dtype=torch.int32, device=dev) if arith == "f16x3" else None
        rgb_map, depth = torch.empty(B, 3, device=dev), torch.empty(B, device=dev)
        weights = torch.empty(B, N, device=dev)
        _lib.check(lib.nerf_normalize_dirs(P(d), B, P(dn), s), "nerf_normalize_dirs")          # render.py:19
        _lib.check(lib.nerf_sample_stratified(P(o), P(dn), B, spec["near"], spec["far"], N,
                                              P(linspace_table(N, dev)), int(spec["perturb"]), P(spec["t_rand"]),
                                              rng_key_at(spec["seed"], spec["ray0"] * N), P(z), None, s),
                   "nerf_sample_stratified")                                                        # :22
        _lib.check(lib.nerf_ray_features_train(P(packed), P(dn), B, P(appd), rows, P(feat), P(encd), s),
                   "nerf_ray_features_train")
        _lib.check(lib.nerf_mlp_forward_train(P(packed), P(o), P(dn), P(z), B, N, P(feat), P(encd), P(rgb), P(sigma),
                                              P(save), P(masks), s), "nerf_mlp_forward_train")      # :49
        _lib.check(lib.nerf_composite(P(rgb), P(sigma), P(z), B, N, P(rgb_map), P(depth), P(weights), s),
                   "nerf_composite")                                                                # :56-80
        ctx.spec = dict(B=B, N=N, packed=packed, packedT=packedT, app=appd, rows=rows, keys=spec["keys"],
                        app_requires_grad=app is not None and app.requires_grad)
        ctx.bufs = (z, rgb, sigma, save, masks)
        ctx.params = params
        ctx.app_in = app
        ctx.mark_non_differentiable(weights, z)
        ctx.set_materialize_grads(False)
        return rgb_map, depth, weights, z

    @staticmethod
    def backward(ctx, g_rgb, g_depth, _gw, _gz):
        lib, s, P = _lib.load(), _lib.stream(), _lib.ptr
        sp = ctx.spec
        z, rgb, sigma, save, masks = ctx.bufs
        B, N = sp["B"], sp["N"]
        M = B * N
        dev = z.device
        if M == 0:
            grads = [torch.zeros_like(p) for p in ctx.params]
            return (None, None if ctx.app_in is None else torch.zeros_like(ctx.app_in), *grads)
        g_rgb = None if g_rgb is None else g_rgb.reshape(B, 3).to(dev, torch.float32).contiguous()
        g_depth = None if g_depth is None else g_depth.reshape(B).to(dev, torch.float32).contiguous()
        dsigma, drgb = torch.empty(M, device=dev), torch.empty(M, 3, device=dev)
        _lib.check(lib.nerf_composite_backward_grad(P(rgb), P(sigma), P(z), P(g_rgb), P(g_depth), B, N, P(dsigma),
                                                    P(drgb), s), "nerf_composite_backward_grad")
        grad = _mlp_backward(sp["packed"], sp["packedT"], save, masks, sigma, rgb, dsigma, drgb, M)
        unused = _COLOUR_KEYS if g_rgb is None else ()
        grads, dapp = _param_grads(sp["keys"], ctx.params, sp["app"], sp["rows"], save, grad, M, N, sp["packed"],
                                   sp["app_requires_grad"] and g_rgb is not None, unused)
        ctx.bufs = ctx.params = None
        return (None, _app_grad(dapp, ctx.app_in), *grads)


class _MLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, app, *params):
        lib, s, P = _lib.load(), _lib.stream(), _lib.ptr
        x, d, M = spec["x"], spec["d"], spec["M"]
        packed, packedT = spec["packed"], spec["packedT"]
        appd, rows = spec["app"], spec["rows"]
        dev = x.device
        feat, encd = torch.empty(M, 256, device=dev), torch.empty(M, 32, device=dev)
        z = torch.zeros(M, 1, device=dev)              # one "ray" per point at z = 0: pts = x + d*0 = x
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
        save = torch.empty(_lib.tile_rows(M), _lib.SAVE_ROW, device=dev)   # tile-major rows
        arith = _lib.get_mlp_arith()
        masks = torch.empty(M, _lib.MASK_ROW, dtype=torch.int32, device=dev) if arith == "f16x3" else None
        if M:
            _lib.check(lib.nerf_ray_features_train(P(packed), P(d), M, P(appd), rows, P(feat), P(encd), s),
                       "nerf_ray_features_train")
            _lib.check(lib.nerf_mlp_forward_train(P(packed), P(x), P(d), P(z), M, 1, P(feat), P(encd), P(rgb),
                                                  P(sigma), P(save), P(masks), s), "nerf_mlp_forward_train")
        ctx.spec = dict(M=M, packed=packed, packedT=packedT, app=appd, rows=rows, keys=spec["keys"],
                        app_requires_grad=app is not None and app.requires_grad)
        ctx.bufs = (rgb, sigma, save, masks)
        ctx.params = params
        ctx.app_in = app
        ctx.set_materialize_grads(False)
        return rgb, sigma.view(M, 1)

    @staticmethod
    def backward(ctx, g_rgb, g_sigma):
        sp = ctx.spec
        rgb, sigma, save, masks = ctx.bufs
        M = sp["M"]
        dev = rgb.device
        drgb = torch.zeros(M, 3, device=dev) if g_rgb is None else g_rgb.reshape(M, 3).to(dev, torch.float32).contiguous()
        dsig = torch.zeros(M, device=dev) if g_sigma is None else g_sigma.reshape(M).to(dev, torch.float32).contiguous()
        if M == 0:
            grads = [torch.zeros_like(p) for p in ctx.params]
            return (None, None if ctx.app_in is None else torch.zeros_like(ctx.app_in), *grads)
        grad = _mlp_backward(sp["packed"], sp["packedT"], save, masks, sigma, rgb, dsig, drgb, M)
        unused = (_COLOUR_KEYS if g_rgb is None else ()) + (_SIGMA_KEYS if g_sigma is None else ())
        grads, dapp = _param_grads(sp["keys"], ctx.params, sp["app"], sp["rows"], save, grad, M, 1, sp["packed"],
                                   sp["app_requires_grad"] and g_rgb is not None, unused)
        ctx.bufs = ctx.params = None
        return (None, _app_grad(dapp, ctx.app_in), *grads)


def volume_render_grad(model, rays_o, rays_d, near, far, n_samples, appearance_embedding, perturb, *, t_rand=None,
                       seed=None, ray_offset=0):
    """The differentiable volume_render (render.py:5-97, coarse): (rgb_map, depth_map, extras)."""
    dev = _lib.device()
    orig = rays_o.shape
    o = rays_o.detach().reshape(-1, 3).to(dev, torch.float32).contiguous()
    d = rays_d.detach().reshape(-1, 3).to(dev, torch.float32).contiguous()
    B, N = o.shape[0], int(n_samples)
    if N < 1:
        raise ValueError(f"volume_render: n_samples={N}")
    if B * N >= 2 ** 31:
        raise ValueError(f"volume_render: {B} rays x {N} samples exceed the training kernels' 2^31 rows")
    app_in = appearance_embedding if uses_appearance(model) else None
    appd, rows = app_rows(None if app_in is None else app_in.detach(), B, dev)
    tr = None
    if perturb and t_rand is not None:
        tr = t_rand.detach().reshape(B, N).to(dev, torch.float32).contiguous()
    if perturb and tr is None and seed is None:
        seed = draw_seed()
    keys, params = model_params(model)
    packed, packedT = packed_pair(model)
    spec = dict(o=o, d=d, B=B, N=N, near=float(near), far=float(far), perturb=bool(perturb), t_rand=tr,
                seed=int(seed or 0), ray0=int(ray_offset), packed=packed, packedT=packedT, app=appd, rows=rows,
                keys=keys)
    rgb_map, depth, weights, z = _RenderFn.apply(spec, app_in, *params)
    out = rays_o.device
    w = weights.unsqueeze(-1)
    if N == 1:      # the reference's per-sample tensors are empty at one sample (render.py:56-58)
        w = w[:, :0]
    extras = {"weights": w.to(out), "z_vals": z.to(out)}
    return rgb_map.reshape(*orig[:-1], 3).to(out), depth.reshape(*orig[:-1], 1).to(out), extras


def nerf_forward_grad(model, x, d, appearance_embedding):
    """The differentiable NeRF.forward (models.py:105-162): rgb (..., 3), sigma (..., 1)."""
    dev = _lib.device()
    lead = x.shape[:-1]
    xs = x.detach().reshape(-1, 3).to(dev, torch.float32).contiguous()
    ds = d.detach().reshape(-1, 3).to(dev, torch.float32).contiguous()
    M = xs.shape[0]
    app_in = appearance_embedding if uses_appearance(model) else None
    appd, rows = app_rows(None if app_in is None else app_in.detach(), M, dev)
    keys, params = model_params(model)
    packed, packedT = packed_pair(model)
    spec = dict(x=xs, d=ds, M=M, packed=packed, packedT=packedT, app=appd, rows=rows, keys=keys)
    rgb, sigma = _MLPFn.apply(spec, app_in, *params)
    return rgb.reshape(*lead, 3).to(x.device), sigma.reshape(*lead, 1).to(x.device)
