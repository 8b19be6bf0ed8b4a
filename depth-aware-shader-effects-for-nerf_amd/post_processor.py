"""Depth-aware post effects on the GPU — the reference's PostProcessor (src/post_processor.py:8-57,
:495-499) for the effects that read the depth map, SURVEY.md §8f row 4.

Same surface: ``PostProcessor()`` with ``effects`` (name -> callable), ``params`` (the reference's
defaults, post_processor.py:33-55), ``current_effect`` and ``apply_effect(image, depth=None)``.
The arithmetic runs in csrc/effects.hip through the C ABI (nerf_effect_fog, nerf_effect_toon);
there is no CPU path.

Effects here: "Original", "Toon Shader" (:64-117), "Fog" (:451-493).  The other twelve effects of
the reference are colour filters that ignore depth (and mostly need cv2, which is absent here);
selecting one raises NotImplementedError naming it.

``image``: uint8 (H,W,3) RGB, a numpy array (as the reference takes) or a torch tensor on the GPU;
``depth``: float (H,W) (Fog also takes (H,W,C) and uses channel 0, as :474-475 do) or None.  The
result has the image's kind: numpy in, numpy out; a device tensor in, a device tensor out.
"""
import numpy as np
import torch

from . import _lib

REFERENCE_ONLY_EFFECTS = ("Color Boost", "Sepia", "Bloom", "Vignette", "Night Vision", "Film Grain",
                          "Pencil Sketch", "Cross Processing", "Posterize", "Neon Glow", "Hologram")


def normalize_depth(depth):
    """run.py:248: (d - min) / (max - min + 1e-6), on the GPU; depth (H,W) float32 (numpy or torch)."""
    lib, dev = _lib.load(), _lib.device()
    as_numpy = isinstance(depth, np.ndarray)
    d = torch.as_tensor(np.ascontiguousarray(depth, np.float32) if as_numpy else depth).to(dev, torch.float32)
    d = d.contiguous()
    out = torch.empty_like(d)
    ws = torch.empty(256, dtype=torch.uint8, device=dev)
    _lib.check(lib.nerf_depth_normalize(_lib.ptr(d), d.numel(), _lib.ptr(out), _lib.ptr(ws), ws.numel(),
                                        _lib.stream()), "nerf_depth_normalize")
    return out.cpu().numpy() if as_numpy else out


def frame_fog(rgb, depth, fog_start=0.1):
    """The CLI's Fog frame straight from the render outputs (nerf_frame_fog): rgb float (H,W,3) in
    [0, 1] -> uint8 by truncation (run.py:233), depth float (H,W) normalised (run.py:248), then Fog
    (post_processor.py:451-493) — one reduction and one per-pixel pass on the GPU instead of a host
    round trip, a normalisation pass and the effect's own reduction.  Bit-identical to
    ``PostProcessor`` Fog on ``normalize_depth(depth)`` and ``(rgb * 255).astype(uint8)``.
    Device tensors in, a uint8 (H,W,3) device tensor out."""
    lib, dev = _lib.load(), _lib.device()
    r = torch.as_tensor(rgb).to(dev, torch.float32).contiguous()
    d = torch.as_tensor(depth).to(dev, torch.float32).contiguous()
    if r.dim() != 3 or r.shape[2] != 3 or tuple(d.shape) != tuple(r.shape[:2]):
        raise ValueError(f"frame_fog: rgb {tuple(r.shape)} must be (H,W,3) and depth {tuple(d.shape)} (H,W)")
    H, W = d.shape
    out = torch.empty(H, W, 3, dtype=torch.uint8, device=dev)
    ws = torch.empty(256, dtype=torch.uint8, device=dev)
    _lib.check(lib.nerf_frame_fog(_lib.ptr(r), _lib.ptr(d), H, W, float(fog_start), _lib.ptr(out), _lib.ptr(ws),
                                  ws.numel(), _lib.stream()), "nerf_frame_fog")
    return out


class PostProcessor:
    """GPU post-processor with the reference's effect names and parameters."""

    def __init__(self):
        self.effects = {
            "Original": self._effect_original,
            "Toon Shader": self._effect_toon,
            "Fog": self._effect_fog,
        }
        self.params = {                                  # post_processor.py:33-55
            "toon_levels": 5,
            "toon_edge_strength": 1.0,
            "edge_threshold": 20,
            "color_saturation": 1.5,
            "bloom_strength": 0.3,
            "bloom_size": 15,
            "vignette_strength": 0.5,
            "fog_density": 5.0,
            "fog_color_r": 200,
            "fog_color_g": 220,
            "fog_color_b": 255,
            "fog_start": 0.1,
            "fog_ray_intensity": 0.5,
            "fog_opacity": 0.8,
            "film_grain_amount": 0.2,
            "sketch_strength": 1.0,
            "posterize_levels": 4,
            "neon_glow_intensity": 0.7,
            "neon_glow_radius": 10,
            "hologram_lines": 50,
            "hologram_intensity": 0.8,
        }
        self.current_effect = "Original"

    # ------------------------------------------------------------------ plumbing
    @staticmethod
    def _inputs(image, depth, allow_channels):
        dev = _lib.device()
        as_numpy = isinstance(image, np.ndarray)
        img = torch.as_tensor(np.ascontiguousarray(image) if as_numpy else image)
        if img.dtype != torch.uint8 or img.dim() != 3 or img.shape[2] != 3:
            raise ValueError(f"PostProcessor: image must be uint8 (H,W,3), got {tuple(img.shape)} {img.dtype}")
        img = img.to(dev).contiguous()
        H, W = img.shape[:2]
        d, stride = None, 1
        if depth is not None:
            d = torch.as_tensor(np.ascontiguousarray(depth, np.float32) if isinstance(depth, np.ndarray) else depth)
            d = d.to(dev, torch.float32).contiguous()
            if d.dim() == 3 and allow_channels:
                stride = d.shape[2]
            elif d.dim() != 2:
                raise ValueError(f"PostProcessor: depth must be (H,W){' or (H,W,C)' if allow_channels else ''}, "
                                 f"got {tuple(d.shape)}")
            if tuple(d.shape[:2]) != (H, W):
                raise ValueError(f"PostProcessor: depth {tuple(d.shape)} does not match image {H}x{W}")
        return img, d, stride, as_numpy

    @staticmethod
    def _workspace(H, W):
        return torch.empty(_lib.load().nerf_effect_workspace_bytes(H, W), dtype=torch.uint8, device=_lib.device())

    # ------------------------------------------------------------------- effects
    def _effect_original(self, image, depth=None):
        """post_processor.py:60-62."""
        return image

    def _effect_fog(self, image, depth=None):
        """post_processor.py:451-493 on the GPU (nerf_effect_fog)."""
        img, d, stride, as_numpy = self._inputs(image, depth, allow_channels=True)
        H, W = img.shape[:2]
        if d is None:
            print("Warning: No depth information for fog effect")      # post_processor.py:467
        out = torch.empty_like(img)
        ws = self._workspace(H, W)
        _lib.check(_lib.load().nerf_effect_fog(_lib.ptr(img), _lib.ptr(d), stride, H, W,
                                               float(self.params.get("fog_start", 0.0)), _lib.ptr(out),
                                               _lib.ptr(ws), ws.numel(), _lib.stream()), "nerf_effect_fog")
        return out.cpu().numpy() if as_numpy else out

    def _effect_toon(self, image, depth=None):
        """post_processor.py:64-117 on the GPU (nerf_effect_toon)."""
        img, d, _, as_numpy = self._inputs(image, depth, allow_channels=False)
        H, W = img.shape[:2]
        out = torch.empty_like(img)
        ws = self._workspace(H, W)
        _lib.check(_lib.load().nerf_effect_toon(_lib.ptr(img), _lib.ptr(d), 1, H, W,
                                                float(self.params.get("toon_levels", 5)),
                                                float(self.params.get("toon_edge_strength", 1.0)), _lib.ptr(out),
                                                _lib.ptr(ws), ws.numel(), _lib.stream()), "nerf_effect_toon")
        return out.cpu().numpy() if as_numpy else out

    def apply_effect(self, image, depth=None):
        """post_processor.py:495-499: the current effect (unknown names return the image)."""
        if self.current_effect in self.effects:
            return self.effects[self.current_effect](image, depth)
        if self.current_effect in REFERENCE_ONLY_EFFECTS:
            raise NotImplementedError(f"PostProcessor: '{self.current_effect}' is a depth-independent colour filter "
                                      f"of the reference that nerfmi does not run on the GPU "
                                      f"(available: {sorted(self.effects)})")
        return image
