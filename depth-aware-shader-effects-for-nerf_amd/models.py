"""NeRF model surface (src/models.py of the reference), computed by libnerfmi.so.

``NeRF`` keeps the reference's module tree, parameter names, shapes and
construction order (src/models.py:58-103), so ``torch.manual_seed(0); NeRF(Config())``
draws the same weights and ``load_state_dict`` accepts the reference's checkpoints
(run.py:363).  Its forward runs the fused PE -> MLP HIP kernel (csrc/mlp16.hip, csrc/mlp.hip)
on weights packed once per parameter version into the MFMA fragment layout (csrc/layout.h).
With gradients enabled and trainable parameters (or an appearance embedding that requires grad)
the forward runs the training kernels instead and is differentiable (autograd.py): the backward
is the MFMA data-gradient chain and weight-gradient reductions of csrc/train.hip.
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib

_APP_DIM = 32


class PositionalEncoding:
    """src/models.py:6-54: [x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(2^(L-1) x)]."""

    def __init__(self, num_frequencies, include_input=True):
        self.num_frequencies = num_frequencies
        self.include_input = include_input

    def output_dim(self, input_dim):
        if self.include_input:
            return input_dim * (1 + 2 * self.num_frequencies)
        return input_dim * 2 * self.num_frequencies

    def __call__(self, x):
        dev = _lib.device()
        dims = x.shape[-1]
        xf = x.reshape(-1, dims).to(dev, torch.float32).contiguous()
        out = torch.empty(xf.shape[0], self.output_dim(dims), device=dev)
        _lib.check(_lib.load().nerf_positional_encoding(_lib.ptr(xf), xf.shape[0], dims, self.num_frequencies,
                                                         int(bool(self.include_input)), _lib.ptr(out),
                                                         _lib.stream()), "nerf_positional_encoding")
        return out.reshape(*x.shape[:-1], out.shape[-1]).to(x.device)


def pack_params(tensors, dev):
    """Pack the 24 state_dict tensors (reference key order) into the fragment layout on `dev`."""
    lib = _lib.load()
    ts = [t.detach().to(dev, torch.float32).contiguous() for t in tensors]
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    packed = torch.empty(lib.nerf_packed_weights_floats(), device=dev)
    _lib.check(lib.nerf_pack_weights(arr, _lib.ptr(packed), _lib.stream()), "nerf_pack_weights")
    return packed


STATE_KEYS = tuple(
    [f"pts_linears.{i}.{p}" for i in range(8) for p in ("weight", "bias")]
    + ["density_head.weight", "density_head.bias", "dir_linear.weight", "dir_linear.bias",
       "appearance_projection.weight", "appearance_projection.bias", "rgb_linear.weight", "rgb_linear.bias"])


APP_KEYS = ("appearance_projection.weight", "appearance_projection.bias")
_APP_SHAPES = ((128, _APP_DIM), (128,))


def state_tensors(sd, dev=None):
    """The 24 packer inputs in STATE_KEYS order from a state_dict.  A model built with
    use_appearance=False has no appearance_projection (models.py:99-103); its two slots are
    zeros, which the kernels never read because such a model ignores the embedding
    (models.py:146)."""
    out = []
    for k in STATE_KEYS:
        if k in sd:
            out.append(sd[k])
        elif k in APP_KEYS:
            out.append(torch.zeros(_APP_SHAPES[APP_KEYS.index(k)], device=dev))
        else:
            raise KeyError(f"state_dict has no {k!r}")
    return out


def uses_appearance(model):
    """models.py:146: the embedding is used only when config.use_appearance is set."""
    cfg = getattr(model, "config", None)
    if cfg is not None:
        return bool(cfg.use_appearance)
    return hasattr(model, "appearance_projection")


def _check_config(config):
    want = dict(hidden_dim=256, num_layers=8, skip_connect_layers=[4], pos_enc_levels=10, dir_enc_levels=4,
                appearance_dim=_APP_DIM)
    bad = {}
    for k, v in want.items():
        got = getattr(config, k)
        if (list(got) if isinstance(v, list) else got) != v:
            bad[k] = got
    if bad:
        raise NotImplementedError(f"nerfmi kernels are built for the reference Config shapes {want}; got {bad}")


class NeRF(nn.Module):
    """src/models.py:57-162 with the forward on the fused HIP MLP."""

    def __init__(self, config):
        super().__init__()
        _check_config(config)
        self.config = config
        self.pos_encoder = PositionalEncoding(config.pos_enc_levels)
        self.dir_encoder = PositionalEncoding(config.dir_enc_levels)
        pos_enc_dim = 3 * (1 + 2 * config.pos_enc_levels)
        dir_enc_dim = 3 * (1 + 2 * config.dir_enc_levels)
        # same construction order as models.py:72-103, so a seeded init draws the same weights
        self.pts_linears = nn.ModuleList()
        self.pts_linears.append(nn.Linear(pos_enc_dim, config.hidden_dim))
        for i in range(1, config.num_layers):
            if i in config.skip_connect_layers:
                self.pts_linears.append(nn.Linear(config.hidden_dim + pos_enc_dim, config.hidden_dim))
            else:
                self.pts_linears.append(nn.Linear(config.hidden_dim, config.hidden_dim))
        self.density_head = nn.Linear(config.hidden_dim, 1)
        self.dir_linear = nn.Linear(config.hidden_dim + dir_enc_dim, config.hidden_dim // 2)
        if config.use_appearance:                                      # models.py:99-103
            self.appearance_projection = nn.Linear(config.appearance_dim, config.hidden_dim // 2)
        self.rgb_linear = nn.Linear(config.hidden_dim // 2, 3)
        self._packed = None
        self._packed_key = None

    # ------------------------------------------------------------------ packed weights
    def packed_weights(self):
        """Device buffer of the MFMA-layout weights; re-packed when any parameter changes."""
        dev = _lib.device()
        sd = self.state_dict()
        key = (dev,) + tuple((sd[k].data_ptr(), sd[k]._version, sd[k].device) for k in STATE_KEYS if k in sd)
        if self._packed is None or self._packed_key != key:
            self._packed = pack_params(state_tensors(sd, dev), dev)
            self._packed_key = key
        return self._packed

    # ------------------------------------------------------------------------ forward
    def forward(self, x, d, appearance_embedding=None):
        """rgb (..., 3), sigma (..., 1) of NeRF.forward (models.py:105-162)."""
        from . import autograd
        if autograd.needs_grad(self, appearance_embedding if self.config.use_appearance else None, x, d):
            return autograd.nerf_forward_grad(self, x, d, appearance_embedding)
        dev = _lib.device()
        lead = x.shape[:-1]
        xs = x.reshape(-1, 3).to(dev, torch.float32).contiguous()
        ds = d.reshape(-1, 3).to(dev, torch.float32).contiguous()
        M = xs.shape[0]
        app, rows = app_rows(appearance_embedding if self.config.use_appearance else None, M, dev)
        return run_mlp(self.packed_weights(), xs, ds, None, M, 1, app, rows, lead, x.device)


def app_rows(app, rows_needed, dev):
    """Appearance tensor and its row count for the C ABI (render.py:33-46, models.py:146-153):
    None -> 0 rows; (32,) or (1,32) -> 1 broadcast row; (R,32) -> R rows."""
    if app is None:
        return None, 0
    a = app.to(dev, torch.float32)
    if a.dim() == 1:
        a = a.unsqueeze(0)
    a = a.reshape(-1, a.shape[-1]).contiguous()
    if a.shape[-1] != _APP_DIM:
        raise ValueError(f"appearance embedding width {a.shape[-1]} != {_APP_DIM}")
    if a.shape[0] == 1:
        return a, 1
    if a.shape[0] != rows_needed:
        raise ValueError(f"appearance embedding has {a.shape[0]} rows for {rows_needed} rays/samples")
    return a, rows_needed


def run_mlp(packed, origins, dirs, z_vals, R, N, app, rows, lead, out_device):
    lib = _lib.load()
    dev = origins.device
    M = R * N
    feat = torch.empty(R, 256, device=dev)
    rgb = torch.empty(M, 3, device=dev)
    sigma = torch.empty(M, 1, device=dev)
    s = _lib.stream()
    _lib.check(lib.nerf_ray_features(_lib.ptr(packed), _lib.ptr(dirs), R, _lib.ptr(app), rows, _lib.ptr(feat), s),
               "nerf_ray_features")
    _lib.check(lib.nerf_mlp_forward(_lib.ptr(packed), _lib.ptr(origins), _lib.ptr(dirs), _lib.ptr(z_vals), R, N,
                                    _lib.ptr(feat), _lib.ptr(rgb), _lib.ptr(sigma), None, 0, s), "nerf_mlp_forward")
    return rgb.reshape(*lead, 3).to(out_device), sigma.reshape(*lead, 1).to(out_device)
