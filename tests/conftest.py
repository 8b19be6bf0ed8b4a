import json
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (runs on the MI355X box)")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def golden_meta():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name)))
    return load


@pytest.fixture(scope="session")
def ref_state(golden_meta):
    """The reference's torch.manual_seed(0); NeRF(Config()) parameters, regenerated and hash-checked."""
    import hashlib
    from oracle import nerf_oracle as O
    st = O.random_state(0)
    h = hashlib.sha256()
    for k in O.STATE_KEYS:
        h.update(st[k].numpy().tobytes())
    assert h.hexdigest() == golden_meta["F0"]["state_sha256"], "weight regeneration drifted from the reference"
    return st


@pytest.fixture(scope="session")
def noapp_state(golden_meta):
    """torch.manual_seed(0); NeRF(config) with use_appearance=False (fixture F8), hash-checked."""
    import hashlib
    from oracle import nerf_oracle as O
    st = O.random_state(0, use_appearance=False)
    assert list(st.keys()) == golden_meta["F8"]["keys"]
    h = hashlib.sha256()
    for k in st:
        h.update(st[k].numpy().tobytes())
    assert h.hexdigest() == golden_meta["F8"]["state_sha256"], "no-appearance weights drifted from the reference"
    return st


@pytest.fixture(scope="session")
def app_vec():
    torch.manual_seed(1)
    return torch.randn(100, 32)[0].clone()


def seeded_uniform(seed, shape, sha=None):
    import hashlib
    torch.manual_seed(seed)
    u = torch.rand(*shape)
    if sha is not None:
        assert hashlib.sha256(u.numpy().tobytes()).hexdigest() == sha, "torch CPU generator drifted"
    return u


def render_h1_f64(state, o, d, app, u, n_samples=64, n_importance=128, chunk=1024, t=None):
    """The oracle's H1 render evaluated in float64 (same expressions and fp32 inputs): the
    reference truth the fp32 paths are measured against.  CPU tensors; (rgb, depth) float64.
    t: the stratified jitter uniforms (perturb=True), None for perturb=False."""
    import torch
    from oracle import nerf_oracle as O
    st64 = {k: v.double() for k, v in state.items()}
    outs = []
    for i in range(0, o.shape[0], chunk):
        r, dd, _ = O.render_rays_h1(st64, o[i:i + chunk].double(), d[i:i + chunk].double(), 2.0, 6.0,
                                    n_samples, n_importance, None if app is None else app.double(),
                                    None if t is None else t[i:i + chunk].double(), u[i:i + chunk].double())
        outs.append((r, dd))
    return torch.cat([a for a, _ in outs]), torch.cat([b for _, b in outs])


def check_no_worse_than_cpu(gpu, cpu, f64, what, factor=1.5):
    """Per value, the relative error of `gpu` against the float64 truth is no worse than the fp32
    CPU oracle's own, in max, p99.9 and median, up to `factor`."""
    eg = ((gpu.double() - f64).abs() / (f64.abs() + 1e-6)).flatten().numpy()
    ec = ((cpu.double() - f64).abs() / (f64.abs() + 1e-6)).flatten().numpy()
    sg = (eg.max(), np.quantile(eg, 0.999), np.median(eg))
    sc = (ec.max(), np.quantile(ec, 0.999), np.median(ec))
    print(f"{what}: rel err vs f64 max/p99.9/median  gpu {sg[0]:.3g} {sg[1]:.3g} {sg[2]:.3g}   "
          f"cpu fp32 {sc[0]:.3g} {sc[1]:.3g} {sc[2]:.3g}")
    for a, b, name in zip(sg, sc, ("max", "p99.9", "median")):
        assert a <= factor * b + 1e-9, (what, name, a, b)
    return sg, sc
