"""ctypes binding of libnerfmi.so (include/nerfmi.h) — the only way nerfmi computes.

There is deliberately no CPU fallback: if the library is missing, or no HIP device is
visible, every compute entry point raises RuntimeError.  PyTorch supplies device memory
and the current HIP stream; all arithmetic happens in the library's HIP kernels.
"""
import ctypes
import os

import torch

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# NERFMI_LIB: an alternative build of the same library (A/B timing of kernel variants on one box)
LIB_PATH = os.environ.get("NERFMI_LIB") or os.path.join(_PKG_DIR, "libnerfmi.so")

_c_float_p = ctypes.c_void_p  # device pointers travel as integers
SAVE_ROW, GRAD_ROW, MASK_ROW = 2400, 2320, 68   # include/nerfmi_train.h NERF_SAVE_ROW, _GRAD_ROW, _MASK_ROW


def tile_rows(M):
    """Rows a tile-major save/grad buffer of M samples holds (include/nerfmi_train.h NERF_TILE_ROWS):
    whole 32-sample blocks."""
    return (M + 31) // 32 * 32


def untile(t, M):
    """A tile-major [tile_rows(M), R] save/grad buffer as the plain [M, R] rows it encodes: element f
    of sample m sits at (m/32)*32R + (f/8)*256 + (m%32)*8 + f%8 (include/nerfmi_train.h)."""
    R = t.shape[1]
    return t.reshape(-1, R // 8, 32, 8).permute(0, 2, 1, 3).reshape(-1, R)[:M]


def tile(x):
    """The inverse of untile: plain [M, R] rows (R % 8 == 0) into a zero-padded tile-major buffer."""
    M, R = x.shape
    out = x.new_zeros(tile_rows(M), R)
    out[:M] = x
    return out.reshape(-1, 32, R // 8, 8).permute(0, 2, 1, 3).reshape(-1, R).contiguous()
_V, _I64 = ctypes.c_void_p, ctypes.c_int64

# name -> (restype, argtypes)
_SIGNATURES = {
    "nerf_last_error": (ctypes.c_char_p, []),
    "nerf_abi_version": (ctypes.c_int, []),
    "nerf_get_rays": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.POINTER(ctypes.c_float),
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_normalize_dirs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_positional_encoding": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_sample_stratified": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double,
                                              ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    "nerf_sample_importance": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    "nerf_sample_importance_merge": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_profile_mlp_begin": (ctypes.c_int, [ctypes.c_int]),
    "nerf_profile_mlp_end": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "nerf_rng_uniforms": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "nerf_packed_weights_floats": (ctypes.c_size_t, []),
    "nerf_set_mlp_arith": (ctypes.c_int, [ctypes.c_int]),
    "nerf_get_mlp_arith": (ctypes.c_int, []),
    "nerf_pack_weights": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_pack_weights_host": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "nerf_ray_features": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "nerf_mlp_forward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "nerf_composite": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "nerf_render_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int, ctypes.c_int]),
    "nerf_render_chunk_rays": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int]),
    "nerf_render_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p]),
    # training (include/nerfmi_train.h)
    "nerf_packed_transposed_floats": (ctypes.c_size_t, []),
    "nerf_pack_weights_transposed": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    "nerf_pack_weights_transposed_host": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "nerf_ray_features_train": (ctypes.c_int, [_V, _V, _I64, _V, _I64, _V, _V, _V]),
    "nerf_mlp_forward_train": (ctypes.c_int, [_V, _V, _V, _V, _I64, ctypes.c_int, _V, _V, _V, _V, _V, _V, _V]),
    "nerf_composite_backward": (ctypes.c_int, [_V, _V, _V, _V, _V, _I64, ctypes.c_int, ctypes.c_float, _V, _V, _V,
                                               _V]),
    "nerf_composite_backward_grad": (ctypes.c_int, [_V, _V, _V, _V, _V, _I64, ctypes.c_int, _V, _V, _V]),
    "nerf_mlp_backward": (ctypes.c_int, [_V, _V, _V, _V, _V, _V, _V, _V, _I64, _V, _V]),
    "nerf_param_grads_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "nerf_param_grads": (ctypes.c_int, [_V, _V, _I64, ctypes.c_int, _V, _I64, _V, ctypes.POINTER(ctypes.c_void_p),
                                        _V, _V, ctypes.c_size_t, _V]),
    "nerf_wgrad_workspace_bytes": (ctypes.c_size_t, [_I64, ctypes.c_int, ctypes.c_int]),
    "nerf_wgrad": (ctypes.c_int, [_V, _I64, ctypes.c_int, _V, _I64, ctypes.c_int, _I64, _I64, _V, _V, ctypes.c_int,
                                  _V, ctypes.c_size_t, _V]),
    "nerf_adam": (ctypes.c_int, [_V, _V, _V, _V, _I64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, _I64, _V]),
    "nerf_train_workspace_bytes": (ctypes.c_size_t, [_I64, ctypes.c_int]),
    "nerf_train_forward": (ctypes.c_int, [_V, _V, _V, _I64, ctypes.c_double, ctypes.c_double, ctypes.c_int, _V,
                                          ctypes.c_int, _V, ctypes.c_uint64, _V, _I64, _V, _V, _V, _V, _V,
                                          ctypes.c_size_t, _V]),
    "nerf_train_backward": (ctypes.c_int, [_V, _V, _V, _V, _I64, ctypes.c_int, _V, _I64,
                                           ctypes.POINTER(ctypes.c_void_p), _V, _V, _V, ctypes.c_size_t, _V]),
    # depth-aware post effects (include/nerfmi.h)
    "nerf_effect_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "nerf_depth_normalize": (ctypes.c_int, [_V, _I64, _V, _V, ctypes.c_size_t, _V]),
    "nerf_effect_fog": (ctypes.c_int, [_V, _V, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_double, _V, _V,
                                       ctypes.c_size_t, _V]),
    "nerf_frame_fog": (ctypes.c_int, [_V, _V, ctypes.c_int, ctypes.c_int, ctypes.c_double, _V, _V, ctypes.c_size_t,
                                      _V]),
    "nerf_effect_toon": (ctypes.c_int, [_V, _V, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, _V,
                                        _V, ctypes.c_size_t, _V]),
}

EXPORTED = tuple(_SIGNATURES)
ABI_VERSION = 11

_lib = None


def load():
    """Load libnerfmi.so (import torch first so its HIP runtime is the one the library binds to)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"nerfmi: {LIB_PATH} is missing — build it with "
                               f"`python -c 'import __graft_entry__ as g; g.build()'` (or make -C {_PKG_DIR})")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.nerf_abi_version() != ABI_VERSION:
            raise RuntimeError(f"nerfmi: {LIB_PATH} has ABI {lib.nerf_abi_version()}, this package needs "
                               f"{ABI_VERSION}; rebuild it")
        _lib = lib
    return _lib


ARITH = {"f32": 0, "f16x3": 1}


def set_mlp_arith(name):
    """Select the MLP's MFMA arithmetic for this process (include/nerfmi.h, nerf_arith):
    "f16x3" (default; split-f16, fp32-accurate) or "f32" (exact f32 products).  Returns the
    previous name."""
    if name not in ARITH:
        raise ValueError(f"nerfmi: unknown MLP arithmetic {name!r}; expected one of {sorted(ARITH)}")
    prev = load().nerf_set_mlp_arith(ARITH[name])
    return {v: k for k, v in ARITH.items()}[prev]


def get_mlp_arith():
    return {v: k for k, v in ARITH.items()}[load().nerf_get_mlp_arith()]


def check(rc, what):
    if rc != 0:
        msg = load().nerf_last_error().decode(errors="replace")
        raise RuntimeError(f"nerfmi: {what} failed (status {rc}): {msg}")


def device():
    """The HIP device all nerfmi work runs on; raises when there is none (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("nerfmi: no HIP device is visible; the render path runs only on the GPU "
                           "(there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def profile_mlp_begin(capacity=4096):
    """Start bracketing every fused-MLP launch with HIP events on its stream (bench.py roofline)."""
    check(load().nerf_profile_mlp_begin(int(capacity)), "nerf_profile_mlp_begin")
    return int(capacity)


def profile_mlp_end(capacity=4096):
    """Stop recording; [(ms, samples)] per MLP launch since profile_mlp_begin."""
    ms = (ctypes.c_float * capacity)()
    samples = (ctypes.c_int64 * capacity)()
    count = ctypes.c_int(0)
    check(load().nerf_profile_mlp_end(ms, samples, capacity, ctypes.byref(count)), "nerf_profile_mlp_end")
    n = min(count.value, capacity)
    return [(float(ms[i]), int(samples[i])) for i in range(n)]
