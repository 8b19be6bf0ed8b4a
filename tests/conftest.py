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
