"""The tile-major save/grad row layout (include/nerfmi_train.h NERF_TILE_ROWS): the host helpers
_lib.tile / _lib.untile agree with the header's element formula and invert each other."""
import torch

from nerfmi import _lib as L


def test_tile_formula_and_round_trip():
    for M, R in [(1, 8), (31, 16), (32, 2400), (33, 2320), (100, 64)]:
        x = torch.arange(M * R, dtype=torch.float32).reshape(M, R)
        t = L.tile(x)
        assert t.shape == (L.tile_rows(M), R)
        flat = t.reshape(-1)
        m = torch.arange(M)[:, None]
        f = torch.arange(R)[None, :]
        idx = (m // 32) * 32 * R + (f // 8) * 256 + (m % 32) * 8 + f % 8
        assert torch.equal(flat[idx], x)
        assert torch.equal(L.untile(t, M), x)
        pad = torch.ones(flat.numel(), dtype=torch.bool)
        pad[idx.reshape(-1)] = False
        assert torch.all(flat[pad] == 0)
