"""nerfmi — MI355X-native NeRF volumetric renderer (import name ``nerfmi``).

Drop-in for the hot path of ByeongKyuPark/Depth-Aware-Shader-Effects-for-NeRF
(src/ray_utils.py, src/models.py, src/render.py): same names, signatures and
state_dict format; every computation runs in libnerfmi.so's HIP kernels for gfx950.
"""
from ._lib import get_mlp_arith, set_mlp_arith
from .config import Config
from .models import NeRF, PositionalEncoding
from .post_processor import PostProcessor
from .ray_utils import get_rays, sample_importance, sample_stratified
from .render import render_rays, volume_render

__all__ = ["Config", "NeRF", "PositionalEncoding", "get_rays", "sample_stratified", "sample_importance",
           "volume_render", "render_rays", "set_mlp_arith", "get_mlp_arith", "PostProcessor"]
