"""The reference-side ctypes binding shown in INTEGRATION.md runs as written (library path
substituted) and agrees with the oracle."""
import os
import re

import pytest
import torch

from conftest import REPO
from oracle import nerf_oracle as O


def stub_source():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(.*?)```", text, re.S).group(1)
    from nerfmi import _lib
    return block.replace('ctypes.CDLL("libnerfmi.so")', f'ctypes.CDLL({_lib.LIB_PATH!r})')


def test_stub_compiles():
    compile(stub_source(), "INTEGRATION.md", "exec")


@pytest.mark.gpu
def test_stub_renders_like_the_oracle(golden, ref_state, app_vec):
    import nerfmi
    ns = {}
    exec(stub_source(), ns)
    model = nerfmi.NeRF(nerfmi.Config())
    model.load_state_dict(ref_state)
    model = model.cuda()
    f1 = golden("f1_get_rays.npz")
    o = torch.from_numpy(f1["chair_o"])[:512]
    d = torch.from_numpy(f1["chair_d"])[:512]
    rgb, depth, ex = ns["volume_render"](model, o.cuda(), d.cuda(), 2.0, 6.0, 64, 64,
                                         appearance_embedding=app_vec.cuda(), perturb=False)
    r_ref, d_ref, _ = O.volume_render(ref_state, o, d, 2.0, 6.0, 64, app_vec)
    assert torch.allclose(rgb.cpu(), r_ref, rtol=1e-4, atol=1e-6)
    assert torch.allclose(depth.cpu(), d_ref, rtol=1e-4, atol=1e-6)
